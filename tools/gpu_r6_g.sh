# Round 6, GPU call G: near-init ring re-checks of the large-K sampler with
# the A searches in LDS (variants/nb3: three kept batch sums; ru4: four
# branch-free rounds; rb10: a 2 x 10 default ring), large-K parity on each,
# then C5 near init / after 30 sweeps against the tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6g; mkdir -p $O
for v in nb3 ru4 rb10; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py -k "large_k or sparse" > $O/parity_$v.log 2>&1 \
    || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6g 0 tree variants/nb3/liblda_mi355x.so variants/ru4/liblda_mi355x.so variants/rb10/liblda_mi355x.so || exit 1
