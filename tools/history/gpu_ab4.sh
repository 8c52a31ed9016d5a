set -o pipefail
cd "$GRAFT_REPO_ROOT"
# parity of every variant library (dense parity subset), then the C4 A/B
for v in variants/*; do
  LDA_MI355X_LIB=$PWD/$v/liblda_mi355x.so timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py -x -q -k "dense" --timeout 300 --timeout-method thread > gpurun_out/pytest_parity_$(basename $v).log 2>&1 || { echo "PARITY $v FAILED"; tail -30 gpurun_out/pytest_parity_$(basename $v).log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/pytest_parity_$(basename $v).log)"
done
CFG=${CFG:-c4} bash tools/gpu_ab.sh
