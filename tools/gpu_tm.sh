set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/test_topic_model_gpu.py tests/test_hyper_gpu.py tests/test_parity_gpu.py -m gpu -q > gpurun_out/pytest_tm.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -80 gpurun_out/pytest_tm.log; exit 1; }
echo "pytest ok"; tail -3 gpurun_out/pytest_tm.log
