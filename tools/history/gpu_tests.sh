# GPU test suite + smoke (each step under its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -x -q -s ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest ok"; grep -E "K=|passed|failed" gpurun_out/pytest_gpu.log | tail -8
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
