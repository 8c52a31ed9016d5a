# Quarter-wave default (K <= 128): the whole -m gpu suite + smoke, C1 A/B
# against the full-wave kernel, then a C2 profile (kernel trace, FETCH, WRITE,
# SQ, LDS/SALU, GRBM) of k_sample_quarter and the C2 bench line reading it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/quarter2; mkdir -p $O profiles/r02
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -60 $O/pytest_gpu.log; exit 1; }
echo "pytest: $(grep -E 'passed|failed' $O/pytest_gpu.log | tail -1)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in 0 2; do
  LDA_DENSE_HALF=$v timeout -k 10 240 python -u bench.py --config c1 --no-cpu-baseline > $O/bench_c1_v$v.log 2>&1 || { echo "BENCH c1 v$v FAILED"; tail -20 $O/bench_c1_v$v.log; exit 1; }
  echo "c1 v$v: $(tail -1 $O/bench_c1_v$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'])")"
done
PASSES="kt fetch write sq lds grbm" LABEL=c2q BENCH_ARGS="--config c2" bash tools/profile.sh > $O/profile_c2q.log 2>&1 || { echo "PROFILE FAILED"; tail -20 $O/profile_c2q.log; exit 1; }
mkdir -p $O/prof_c2q && cp gpurun_out/prof_c2q/summary_*.json $O/prof_c2q/ && cp gpurun_out/prof_c2q/*kernel_stats.csv $O/prof_c2q/ 2>/dev/null
python3 tools/make_traffic.py gpurun_out/prof_c2q "k_sample_quarter<8, 4, false>" 20000000 c2 $O/traffic_c2.json 128 > /dev/null || { echo "TRAFFIC FAILED"; exit 1; }
cp $O/traffic_c2.json profiles/r02/traffic_c2.json
python3 -c "import json;t=json.load(open('$O/traffic_c2.json'));print('c2', round(t['bytes_per_token'],1),'B/tok', {k:round(v,1) for k,v in t.get('per_token',{}).items()}, 'clk', round(t.get('effective_clock_ghz',0),3))"
for b in 0 30; do
  timeout -k 10 240 python bench.py --config c2 --burnin $b --no-cpu-baseline > $O/bench_c2_b$b.log 2>&1 || { echo "BENCH c2 FAILED"; tail -5 $O/bench_c2_b$b.log; exit 1; }
  tail -1 $O/bench_c2_b$b.log > $O/bench_c2_b$b.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_c2_b$b.jsonl').read());r=d['roofline'];i=r.get('issue') or {};print('c2 b$b', round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],3),'traffic_frac',r.get('traffic_frac'),'issue',i.get('binding'),i.get('frac'))"
done
