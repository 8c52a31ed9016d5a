# Round 6, GPU call V: the large-K sampler with its kernel-argument reads and
# count atomics in their own address spaces (variants/gas, -DSB_GLOBAL_AS=1:
# no FLAT instruction left, so the waitcnt pass waits for each prefetched row
# by count -- vmcnt(14..19) -- instead of vmcnt(0) at every token): parity,
# then C5 near init / after 30 sweeps against the tree, both orders; second
# run adds variants/gat (-DSB_GLOBAL_AS=2: only the pointers' accesses global,
# the kernel-argument reads stay FLAT loads).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6v; mkdir -p $O
for v in gas gat; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_parity_random_gpu.py -k "large_k or sparse or random" \
    > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6v/a 0 tree variants/gat/liblda_mi355x.so variants/gas/liblda_mi355x.so || exit 1
bash tools/gpu_r5_c5ab.sh r6v/b 0 variants/gas/liblda_mi355x.so variants/gat/liblda_mi355x.so tree || exit 1
