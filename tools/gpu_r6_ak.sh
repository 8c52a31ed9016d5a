# Round 6, GPU call AK: the LDS batch size re-checked on the final sampler
# (variants/lb3, lb5, lb6: -DSB_LDS_BATCH=3/5/6 against the tree's 4):
# parity, then C5 near init / after 30 sweeps, both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ak; mkdir -p $O
for v in lb3 lb5 lb6; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_random_gpu.py -k "large_k or sparse or random" \
    > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6ak/a 0 tree variants/lb3/liblda_mi355x.so variants/lb5/liblda_mi355x.so variants/lb6/liblda_mi355x.so || exit 1
bash tools/gpu_r5_c5ab.sh r6ak/b 0 variants/lb6/liblda_mi355x.so variants/lb5/liblda_mi355x.so variants/lb3/liblda_mi355x.so tree || exit 1
