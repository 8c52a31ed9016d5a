# Full parity file for the in-tree library and every variant, then the A/B on CFG (default c5).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_default.log 2>&1 || { echo "PARITY default FAILED"; tail -30 gpurun_out/pytest_parity_default.log; exit 1; }
echo "default: $(tail -1 gpurun_out/pytest_parity_default.log)"
for v in variants/*; do
  LDA_MI355X_LIB=$PWD/$v/liblda_mi355x.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_$(basename $v).log 2>&1 || { echo "PARITY $v FAILED"; tail -30 gpurun_out/pytest_parity_$(basename $v).log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_parity_$(basename $v).log)"
done
CFG=${CFG:-c5} bash tools/gpu_ab.sh
