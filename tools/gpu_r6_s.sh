# Round 6, GPU call S: the batched LDS reads as the default (SB_LDS_BATCH 4 +
# SB_TOKEN_LGKM0): parity on the tree, a second batch of 4 / 2 rounds
# (variants/lb44, lb42) A/B against it, then the tree's C5 profiles near
# init and after 30 sweeps (traffic records for the new machine code).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_parity_gpu.py tests/test_parity_random_gpu.py tests/test_exchange_gpu.py -k "large_k or sparse or random or exchange" \
  > $O/parity_tree.log 2>&1 || { tail -20 $O/parity_tree.log; exit 1; }
echo "tree $(tail -1 $O/parity_tree.log)"
for v in lb44 lb42; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_random_gpu.py -k "large_k or sparse or random" \
    > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6s/a 0 tree variants/lb44/liblda_mi355x.so variants/lb42/liblda_mi355x.so || exit 1
bash tools/gpu_r5_c5ab.sh r6s/b 0 variants/lb42/liblda_mi355x.so variants/lb44/liblda_mi355x.so tree || exit 1
LABEL=r6_c5n BENCH_ARGS="--config c5" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
BURNIN=30 LABEL=r6_c5n_b30 BENCH_ARGS="--config c5" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
