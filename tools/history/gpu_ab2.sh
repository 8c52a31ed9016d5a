# Parity of the in-tree library, then the A/B bench over variants (CFG, BURNINS, SAMPLER env).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_ab.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/pytest_parity_ab.log; exit 1; }
tail -1 gpurun_out/pytest_parity_ab.log
bash tools/gpu_ab.sh
