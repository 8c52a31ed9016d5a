# Round 4 evidence on the tree's library: rocprofv3 passes of the bench
# commands themselves (same warm-up / burn-in / timed window; the summaries
# skip the untimed dispatches), the traffic files bench.py reads
# (profiles/r04/traffic_<label>.json), and the bench lines that carry them.
#   bash tools/gpu_r4_evidence.sh OUT "label kernel tokens K burnin args..." ... 
# Every step under its own timeout; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
mkdir -p $O profiles/r04
export TMPDIR=/tmp
for spec in "$@"; do
  set -- $spec
  L=$1; KN=$2; TOK=$3; K=$4; BI=$5; shift 5
  KN=${KN//\~/ }
  BURNIN=$BI PASSES="kt fetch write sq lds grbm" LABEL=$L BENCH_ARGS="$*" bash tools/profile.sh > $O/profile_$L.log 2>&1 || { echo "PROFILE $L FAILED"; tail -20 $O/profile_$L.log; exit 1; }
  mkdir -p $O/prof_$L && cp gpurun_out/prof_$L/summary_*.json $O/prof_$L/ && cp gpurun_out/prof_$L/*kernel_stats.csv $O/prof_$L/ 2>/dev/null
  python3 tools/make_traffic.py gpurun_out/prof_$L "$KN" $TOK "$L" $O/traffic_$L.json $K $BI > /dev/null || { echo "TRAFFIC $L FAILED"; exit 1; }
  cp $O/traffic_$L.json profiles/r04/traffic_$L.json
  timeout -k 10 900 python bench.py --burnin $BI --no-cpu-baseline "$@" > $O/bench_$L.log 2>&1 || { echo "BENCH $L FAILED"; tail -5 $O/bench_$L.log; exit 1; }
  tail -1 $O/bench_$L.log > $O/bench_$L.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$L.jsonl').read());r=d['roofline'];t=json.load(open('$O/traffic_$L.json'));print('$L', round(d['value']/1e9,4),'Gtok/s kernel',round(r['kernel_ms_timed_region'],3),'ms frac',round(r['frac'],3),'traffic_frac',r.get('traffic_frac'),'B/token',round(t['bytes_per_token'],1),'write B/token',round(t['WRITE_SIZE_KiB']*1024/t['tokens_per_launch'],1))"
done
