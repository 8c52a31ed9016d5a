# Round 3, step Y: the default workload and C3 after 30 burn-in sweeps (the
# tree's library), for DESIGN §0's after-burn-in column.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3y; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms kernel',round(r['kernel_ms_timed_region'],3),'frac',round(r['frac'],3))"; }
for cfg in c4 c3 c2; do
  timeout -k 10 900 python bench.py --no-cpu-baseline --config $cfg --burnin 30 > $O/bench_${cfg}_b30.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 $O/bench_${cfg}_b30.log; exit 1; }
  tail -1 $O/bench_${cfg}_b30.log > $O/bench_${cfg}_b30.jsonl
  line $O/bench_${cfg}_b30.jsonl "$cfg b30"
done
