# Round 6, GPU call R: the batched LDS reads again, with an lgkmcnt(0) at the
# end of every token (-DSB_TOKEN_LGKM0=1: the waitcnt pass had carried a rare
# path's pending LDS write into the next token as an lgkmcnt(0) between the
# batch's first reads and the rest): variants tw (the tree + the wait), lb4w,
# lb6w, lb12w, lb4, lb12; parity on each, then C5 near init / after 30 sweeps
# against the tree, twice in opposite orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6r; mkdir -p $O
V="tw lb4w lb6w lb12w lb12"
for v in $V; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_random_gpu.py -k "large_k or sparse or random" \
    > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
L=""; for v in $V lb4; do L="$L variants/$v/liblda_mi355x.so"; done
bash tools/gpu_r5_c5ab.sh r6r/a 0 tree $L || exit 1
R=""; for v in lb4 lb12 lb12w lb6w lb4w tw; do R="$R variants/$v/liblda_mi355x.so"; done
bash tools/gpu_r5_c5ab.sh r6r/b 0 $R tree || exit 1
