# Round 6, GPU call A: the whole GPU suite on the tree, then the A-search LDS
# variant (variants/apick, -DSB_APICK_LDS=1): large-K parity on it and the C5
# lines near init / after 30 sweeps against the tree.  Stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6a; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
LDA_MI355X_LIB=variants/apick/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread -m gpu tests/test_parity_gpu.py -k "large_k or sparse" > $O/apick_parity.log 2>&1 \
  || { tail -20 $O/apick_parity.log; exit 1; }
tail -1 $O/apick_parity.log
bash tools/gpu_r5_c5ab.sh r6a 0 tree variants/apick/liblda_mi355x.so variants/nodelta/liblda_mi355x.so || exit 1
# the C2 / C3 lines (tree), then the C4 profile passes on the shipped dense kernel
for cfg in c2 c3; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline --no-estimate > $O/bench_$cfg.log 2>&1 || { tail -5 $O/bench_$cfg.log; exit 1; }
  tail -c 400 $O/bench_$cfg.log; echo
done
LABEL=r6_c4 PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
