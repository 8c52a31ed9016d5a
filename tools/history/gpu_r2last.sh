# Last round-2 evidence on the library in the tree: C2 (quarter-wave) PMC
# passes with its traffic file, the C4 kernel trace, then the default bench
# line and C2 reading them.  Everything under gpurun_out/last/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/last; mkdir -p $O profiles/r02
export TMPDIR=/tmp
PASSES="kt fetch write sq lds grbm" LABEL=c2 BENCH_ARGS="--config c2" bash tools/profile.sh > $O/profile_c2.log 2>&1 || { echo "PROFILE c2 FAILED"; tail -20 $O/profile_c2.log; exit 1; }
mkdir -p $O/prof_c2 && cp gpurun_out/prof_c2/summary_*.json $O/prof_c2/ && cp gpurun_out/prof_c2/*kernel_stats.csv $O/prof_c2/ 2>/dev/null
python3 tools/make_traffic.py gpurun_out/prof_c2 "k_sample_quarter<8, 4, false>" 20000000 c2 $O/traffic_c2.json 128 > /dev/null || { echo "TRAFFIC FAILED"; exit 1; }
cp $O/traffic_c2.json profiles/r02/traffic_c2.json
PASSES="kt" LABEL=c4 BENCH_ARGS="--config c4" bash tools/profile.sh > $O/profile_c4.log 2>&1 || { echo "PROFILE c4 FAILED"; tail -20 $O/profile_c4.log; exit 1; }
mkdir -p $O/prof_c4 && cp gpurun_out/prof_c4/summary_*.json $O/prof_c4/ && cp gpurun_out/prof_c4/*kernel_stats.csv $O/prof_c4/ 2>/dev/null
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { echo "BENCH FAILED"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log > $O/bench_default.jsonl
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > $O/bench_c2.log 2>&1 || { echo "BENCH c2 FAILED"; tail -5 $O/bench_c2.log; exit 1; }
tail -1 $O/bench_c2.log > $O/bench_c2.jsonl
for f in $O/bench_*.jsonl; do
  python3 -c "import json;d=json.loads(open('$f').read());r=d['roofline'];i=r.get('issue') or {};print('$f', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms frac',round(r['frac'],3),'traffic_frac',r.get('traffic_frac'),'issue',i.get('binding'),i.get('frac'), r.get('kernel'))"
done
grep -h "k_sample" $O/prof_c4/*kernel_stats.csv $O/prof_c2/*kernel_stats.csv | cut -c1-200
