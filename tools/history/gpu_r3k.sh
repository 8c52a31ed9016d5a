# Round 3, step K: the tree's library (large-K variant A as default, device
# beta for graph sweeps, one statistics fetch per optimisation): every GPU
# test, the reference-scale runs, the estimate() overhead split, C5 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3k; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs.log 2>&1 || { echo "REFRUNS FAILED"; tail -5 $O/reference_runs.log; exit 1; }
cat $O/reference_runs.log
timeout -k 10 300 python tools/estimate_overhead.py > $O/est_overhead.json 2> $O/est_overhead.err || { echo "OVERHEAD FAILED"; tail -5 $O/est_overhead.err; exit 1; }
cat $O/est_overhead.json
for b in 0 30; do
  timeout -k 10 600 python bench.py --no-cpu-baseline --config c5 --burnin $b > $O/bench_c5_b$b.log 2>&1 || { echo "BENCH c5 $b FAILED"; tail -5 $O/bench_c5_b$b.log; exit 1; }
  tail -1 $O/bench_c5_b$b.log > $O/bench_c5_b$b.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_c5_b$b.jsonl').read());r=d['roofline'];print('c5 b$b', round(d['value']/1e9,4),'Gtok/s kernel',round(r['kernel_ms_timed_region'],2),'ms')"
done
