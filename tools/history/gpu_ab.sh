# A/B: bench for the in-tree library and each variants/*/ library (CFG, BURNIN env)
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
CFG=${CFG:-c4}
for b in ${BURNINS:-0}; do
for v in default variants/*/liblda_mi355x.so; do
  v=${v%/liblda_mi355x.so}
  if [ "$v" = default ]; then unset LDA_MI355X_LIB; else export LDA_MI355X_LIB=$PWD/$v/liblda_mi355x.so; fi
  n=$(basename $v)
  timeout -k 10 600 python bench.py --config $CFG ${SAMPLER:+--sampler $SAMPLER} --burnin $b --no-cpu-baseline --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab_${n}_b$b.log 2>&1 || { echo "$n FAILED"; tail -5 gpurun_out/ab_${n}_b$b.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/ab_${n}_b$b.log').read().strip().splitlines()[-1]);print('$n burnin $b', round(d['value']/1e9,4), 'Gtok/s', round(d['roofline']['kernel_ms_timed_region'],3), 'ms')"
done
done
