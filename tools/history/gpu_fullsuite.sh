# The whole -m gpu suite (the driver's round-end command) with durations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/pytest_gpu_full.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -22 gpurun_out/pytest_gpu_full.log
