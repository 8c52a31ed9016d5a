# Round 3, step R: the word-ordered z copy for the quarter-wave sampler's
# recount sweeps (the sampler stores a changed token's topic at its position
# in the recount order; the recount streams it instead of gathering z through
# perm): the recount / exchange / config parity tests, then C2 (and C1) at
# burn-in 0 with LDA_ZW=0 / 1, two repeats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3r; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_recount_gpu.py tests/test_exchange_gpu.py \
  tests/test_configs_gpu.py tests/test_graph_gpu.py tests/test_parity_gpu.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms recount', r.get('recount_ms_timed_region'))"; }
for rep in 1 2; do
  for zw in 0 1; do
    LDA_ZW=$zw timeout -k 10 600 python bench.py --no-cpu-baseline --config c2 > $O/bench_c2_zw${zw}_$rep.log 2>&1 || { echo "BENCH c2 zw$zw FAILED"; tail -5 $O/bench_c2_zw${zw}_$rep.log; exit 1; }
    tail -1 $O/bench_c2_zw${zw}_$rep.log > $O/bench_c2_zw${zw}_$rep.jsonl
    line $O/bench_c2_zw${zw}_$rep.jsonl "c2 zw$zw rep$rep"
  done
done
