# Round 6, GPU call F: 20 waves per CU for the large-K sampler (SB_ND8: byte
# document counts, two 10-wave blocks per CU, <= 96 VGPRs by a leaner ring):
# variants/nd8a (rings 2 x 8 / 2 x 6, batches of 2), variants/nd8b (2 x 10 /
# 3 x 6).  Short-document parity on each (the byte counts hold <= 255), then
# C5 near init / after 30 sweeps against the tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6f; mkdir -p $O
for v in tree nd8a nd8b; do
  if [ $v = tree ]; then L=""; else L=variants/$v/liblda_mi355x.so; fi
  LDA_MI355X_LIB=$L timeout -k 10 300 python -u tools/parity_short_docs.py > $O/parity_$v.log 2>&1 || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
bash tools/gpu_r5_c5ab.sh r6f 0 tree variants/nd8a/liblda_mi355x.so variants/nd8b/liblda_mi355x.so || exit 1
