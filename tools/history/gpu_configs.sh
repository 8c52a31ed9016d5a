set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in c2 c3; do
  for smp in dense sparse; do
    timeout -k 10 600 python bench.py --config $cfg --sampler $smp --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_${cfg}_${smp}.log 2>&1 || { echo BENCH $cfg $smp FAILED; tail -20 gpurun_out/bench_${cfg}_${smp}.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/bench_${cfg}_${smp}.log').read().strip().splitlines()[-1]);print('$cfg $smp', round(d['value']/1e9,3), 'Gtok/s', d['roofline']['kernel'], 'frac', round(d['roofline']['frac'],3))"
  done
done
