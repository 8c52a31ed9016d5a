# Round 6, GPU call AM: a new document's counts from the chunk registers
# (variants/dr, -DSB_DOC_REGS=1): parity (large-K, sparse,
# random and the large-K perplexity-free A-part cases), then C5 near init /
# after 30 sweeps against the tree, both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6am; mkdir -p $O
for v in dr; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_random_gpu.py tests/test_fullsize_gpu.py -k "large_k or sparse or random or c5" \
    > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6am/a 0 tree variants/dr/liblda_mi355x.so || exit 1
bash tools/gpu_r5_c5ab.sh r6am/b 0 variants/dr/liblda_mi355x.so tree || exit 1
