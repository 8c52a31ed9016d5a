# Parity + small corpora + C4/C2 bench lines after the fused apply / range-floor change.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "not perplexity" > gpurun_out/pytest_apply.log 2>&1 || { echo "PYTEST FAILED"; tail -40 gpurun_out/pytest_apply.log; exit 1; }
tail -1 gpurun_out/pytest_apply.log
timeout -k 10 300 python tools/small_corpus.py 0 > gpurun_out/small_corpus2.log 2>&1 || { echo SMALL FAILED; tail -20 gpurun_out/small_corpus2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/small_corpus2.log
for cfg in c4 c2; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline > gpurun_out/bench_apply_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 gpurun_out/bench_apply_$cfg.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_apply_$cfg.log').read().strip().splitlines()[-1]);print('$cfg', round(d['value']/1e9,4), 'Gtok/s', round(d['ms_per_step'],3), 'ms/step', round(d['roofline']['kernel_ms_timed_region'],3), 'ms kernel')"
done
timeout -k 10 600 python bench.py --config c2 --tokens-per-range 256 --no-cpu-baseline > gpurun_out/bench_apply_c2_256.log 2>&1 && python -c "import json;d=json.loads(open('gpurun_out/bench_apply_c2_256.log').read().strip().splitlines()[-1]);print('c2 tpr256', round(d['value']/1e9,4), 'Gtok/s', round(d['ms_per_step'],3), 'ms/step')"
