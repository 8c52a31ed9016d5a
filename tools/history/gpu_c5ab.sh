# C5 large-K kernel A/B: parity (sparse + large-K tests) of the in-tree library
# and every variant, then the C5 bench for each at burn-in 0 and 30.
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default variants/*/; do
  v=${v%/}; n=$(basename $v)
  [ "$n" = src ] && continue
  if [ "$v" = default ]; then unset LDA_MI355X_LIB; else export LDA_MI355X_LIB=$PWD/$v/liblda_mi355x.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -k "sparse or large or infer" --timeout 200 --timeout-method thread > gpurun_out/c5ab_parity_$n.log 2>&1 || { echo "PARITY $n FAILED"; tail -30 gpurun_out/c5ab_parity_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/c5ab_parity_$n.log)"
done
unset LDA_MI355X_LIB
timeout -k 10 300 python -u -m pytest tests/test_fullsize_gpu.py -x -q -k c5 --timeout 200 --timeout-method thread > gpurun_out/c5ab_full.log 2>&1 || { echo "FULLSIZE FAILED"; tail -30 gpurun_out/c5ab_full.log; exit 1; }
echo "fullsize c5: $(tail -1 gpurun_out/c5ab_full.log)"
CFG=c5 BURNINS="${BURNINS:-0 30}" bash tools/gpu_ab.sh
