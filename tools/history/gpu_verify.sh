# Full GPU check of the tree as it stands: every -m gpu test, smoke, default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LABEL=${LABEL:-verify}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$LABEL.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_gpu_$LABEL.log; exit 1; }
echo "pytest ok"; tail -2 gpurun_out/pytest_gpu_$LABEL.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$LABEL.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke_$LABEL.log; exit 1; }
tail -1 gpurun_out/smoke_$LABEL.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$LABEL.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench_$LABEL.log; exit 1; }
tail -1 gpurun_out/bench_$LABEL.log
