# C2 (K = 128, C = 2) scalar/vector balance A/B: parity of each library on the
# dense tests, then bench lines for CFGS (default c2 c1) at burn-in 0 and 30.
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for v in default variants/*/liblda_mi355x.so; do
  v=${v%/liblda_mi355x.so}; n=$(basename $v)
  if [ "$v" = default ]; then unset LDA_MI355X_LIB; else export LDA_MI355X_LIB=$PWD/$v/liblda_mi355x.so; fi
  [ "$v" != default ] && [ -n "$SKIP_VARIANT_PARITY" ] && continue
  timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -x -q -k "${PARITY_K:-dense and not half}" --timeout 200 --timeout-method thread > gpurun_out/c2ab_parity_$n.log 2>&1 || { echo "PARITY $n FAILED"; tail -30 gpurun_out/c2ab_parity_$n.log; exit 1; }
  echo "$n parity: $(tail -1 gpurun_out/c2ab_parity_$n.log)"
done
unset LDA_MI355X_LIB
for cfg in ${CFGS:-c2 c1}; do
  mkdir -p gpurun_out/ab_$cfg
  CFG=$cfg BURNINS="${BURNINS:-0 30}" bash tools/gpu_ab.sh || exit 1
  mv gpurun_out/ab_*_b*.log gpurun_out/ab_$cfg/
done
