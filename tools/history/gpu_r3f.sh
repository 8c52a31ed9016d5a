# Round 3, step F: every -m gpu test and smoke on the tree's library, then the
# reference-scale estimate() runs (src/cmu, src/cmu_ron settings end to end,
# the per-iteration breakdown) and the C1 bench line.  Output: gpurun_out/r3f/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3f; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -v --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
grep -E "^K=|rel diff|median" $O/pytest_gpu.log | head -10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs.log 2>&1 || { echo "REFRUNS FAILED"; tail -5 $O/reference_runs.log; exit 1; }
cat $O/reference_runs.log
timeout -k 10 300 python tools/estimate_overhead.py > $O/est_overhead.json 2> $O/est_overhead.err || { echo "OVERHEAD FAILED"; tail -5 $O/est_overhead.err; exit 1; }
cat $O/est_overhead.json
timeout -k 10 300 python bench.py --config c1 --no-cpu-baseline > $O/bench_c1.log 2>&1 || { echo "BENCH c1 FAILED"; tail -5 $O/bench_c1.log; exit 1; }
tail -1 $O/bench_c1.log | cut -c1-300
