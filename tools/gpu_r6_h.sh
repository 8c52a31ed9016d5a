# Round 6, GPU call H: more branch-free register rounds in the large-K
# sampler (SB_RU 4 / 5 / 6 against the tree's 2): large-K parity on each, then
# C5 near init / after 30 sweeps, the whole A/B twice.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6h; mkdir -p $O
for v in ru5 ru6; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py -k "large_k or sparse" > $O/parity_$v.log 2>&1 \
    || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6h 0 tree variants/ru4/liblda_mi355x.so variants/ru5/liblda_mi355x.so variants/ru6/liblda_mi355x.so || exit 1
bash tools/gpu_r5_c5ab.sh r6h2 0 variants/ru6/liblda_mi355x.so variants/ru5/liblda_mi355x.so variants/ru4/liblda_mi355x.so tree || exit 1
