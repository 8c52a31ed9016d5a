set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_ab.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/pytest_parity_ab.log; exit 1; }
tail -1 gpurun_out/pytest_parity_ab.log
CFG=c3 bash tools/gpu_ab.sh && CFG=c4 bash tools/gpu_ab.sh
