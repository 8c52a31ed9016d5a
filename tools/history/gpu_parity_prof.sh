# Parity of the in-tree library + SQ instruction counters of the dense kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_pp.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/pytest_parity_pp.log; exit 1; }
tail -1 gpurun_out/pytest_parity_pp.log
PASSES="sq lds" LABEL=${LABEL:-pp} bash tools/profile.sh
