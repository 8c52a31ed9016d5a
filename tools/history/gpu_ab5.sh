# Parity of the in-tree library and of every variant (dense subset), then the A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_default.log 2>&1 || { echo "PARITY default FAILED"; tail -30 gpurun_out/pytest_parity_default.log; exit 1; }
echo "default: $(tail -1 gpurun_out/pytest_parity_default.log)"
bash tools/gpu_ab4.sh
