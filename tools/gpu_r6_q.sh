# Round 6, GPU call Q: the large-K sampler's register rounds with their LDS
# reads issued as one batch (variants/lb2, lb4, lb6: -DSB_LDS_BATCH=2/4/6):
# large-K parity on each, then C5 near init / after 30 sweeps against the
# tree, the whole A/B twice in opposite orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q; mkdir -p $O
for v in lb2 lb4 lb6; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_random_gpu.py -k "large_k or sparse or random" \
    > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6q/a 0 tree variants/lb2/liblda_mi355x.so variants/lb4/liblda_mi355x.so variants/lb6/liblda_mi355x.so || exit 1
bash tools/gpu_r5_c5ab.sh r6q/b 0 variants/lb6/liblda_mi355x.so variants/lb4/liblda_mi355x.so variants/lb2/liblda_mi355x.so tree || exit 1
