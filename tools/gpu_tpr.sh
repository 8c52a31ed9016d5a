set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in ${CFGS:-c4}; do
for tpr in ${TPRS:-0 1500 3000 12000}; do
  timeout -k 10 600 python bench.py --config $cfg --tokens-per-range $tpr --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/tpr_${cfg}_$tpr.log 2>&1 || { echo "$tpr FAILED"; tail -5 gpurun_out/tpr_${cfg}_$tpr.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/tpr_${cfg}_$tpr.log').read().strip().splitlines()[-1]);print('$cfg tpr $tpr', round(d['value']/1e9,4), 'Gtok/s', round(d['roofline']['kernel_ms_timed_region'],3), 'ms')"
done
done
