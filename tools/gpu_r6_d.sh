# Round 6, GPU call D: where the large-K sampler's delta atomics cost least
# (variants/dz, -DSB_X_DELTA_KERNEL=1: the sampler without them, the count
# changes made right by k_delta_from_z after the pass; plain-sweep parity on
# it first) and two ring re-checks with the A searches in LDS (variants/rs8:
# short ring 3 x 8; variants/ru3: 3 branch-free rounds), C5 near init and
# after 30 sweeps against the tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6d; mkdir -p $O
for v in dz rs8 ru3; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py -k "large_k_sparse_bit_exact" > $O/parity_$v.log 2>&1 \
    || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6d 0 tree variants/dz/liblda_mi355x.so variants/rs8/liblda_mi355x.so variants/ru3/liblda_mi355x.so || exit 1
