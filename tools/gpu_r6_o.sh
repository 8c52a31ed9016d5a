# Round 6, GPU call O: the LLVM AMDGPU scheduler strategies (variants/sch_*,
# -mllvm --amdgpu-sched-strategy=max-ilp / max-memory-clause / iterative-ilp /
# iterative-minreg) on the whole kernel file: parity on each (large-K, sparse
# and dense sweeps), then C5 near init / after 30 sweeps and the C4 shard
# line against the tree.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6o; mkdir -p $O
for v in sch_mxilp sch_mxmc sch_itilp sch_itmr; do
  LDA_MI355X_LIB=variants/$v/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
    --timeout-method thread -m gpu tests/test_parity_gpu.py -k "large_k or sparse or sweeps_bit_exact" > $O/parity_$v.log 2>&1 \
    || { tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
for lib in tree variants/sch_mxilp/liblda_mi355x.so variants/sch_mxmc/liblda_mi355x.so \
           variants/sch_itilp/liblda_mi355x.so variants/sch_itmr/liblda_mi355x.so; do
  n=$(basename $(dirname $lib)); [ "$lib" = "tree" ] && n=tree
  env_lib=""; [ "$lib" != "tree" ] && env_lib="LDA_MI355X_LIB=$lib"
  env $env_lib timeout -k 10 400 python bench.py --config c4shard --no-cpu-baseline --no-estimate --dropin-steps 0 \
    > $O/c4s_$n.log 2>&1 || { echo "BENCH c4s $n FAILED"; tail -5 $O/c4s_$n.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c4s_$n.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$n c4shard', round(d['value']/1e9,4),'Gtok/s kernel ms',round(r['kernel_ms_timed_region'],3))"
done
bash tools/gpu_r5_c5ab.sh r6o/c5 0 tree variants/sch_mxilp/liblda_mi355x.so variants/sch_mxmc/liblda_mi355x.so \
  variants/sch_itilp/liblda_mi355x.so variants/sch_itmr/liblda_mi355x.so
