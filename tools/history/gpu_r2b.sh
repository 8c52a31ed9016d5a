# Round-2 step B: the JNI harness test, the chip's issue peaks, PMC profiles
# (kernel trace, FETCH, WRITE, SQ instruction mix, GRBM clock) of the sampler
# at C4 / C2 / C3 / C5, the bench lines that read them, and the cost of the
# hyperparameter optimisation at the C4 shard.  Everything under gpurun_out/r2b/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2b; mkdir -p $O profiles/r02
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_jni_harness_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_jni.log 2>&1 \
  || { echo "JNI HARNESS FAILED"; tail -40 $O/pytest_jni.log; exit 1; }
echo "jni: $(tail -1 $O/pytest_jni.log)"
timeout -k 10 120 ./tools/bin/issue_peak > $O/issue_peak.json 2> $O/issue_peak.log || { echo ISSUE_PEAK FAILED; cat $O/issue_peak.log; exit 1; }
cat $O/issue_peak.json; cp $O/issue_peak.json profiles/r02/issue_peak.json
prof() {  # cfg kernel tokens K
  local cfg=$1 kern=$2 tok=$3 K=$4
  PASSES="kt fetch write sq lds grbm" LABEL=$cfg BENCH_ARGS="--config $cfg" bash tools/profile.sh > $O/profile_$cfg.log 2>&1 || { echo "PROFILE $cfg FAILED"; tail -20 $O/profile_$cfg.log; return 1; }
  mkdir -p $O/prof_$cfg && cp gpurun_out/prof_$cfg/summary_*.json $O/prof_$cfg/ && cp gpurun_out/prof_$cfg/*kernel_stats.csv $O/prof_$cfg/ 2>/dev/null
  python3 tools/make_traffic.py gpurun_out/prof_$cfg "$kern" $tok $cfg $O/traffic_$cfg.json $K > /dev/null || { echo "TRAFFIC $cfg FAILED"; return 1; }
  cp $O/traffic_$cfg.json profiles/r02/traffic_$cfg.json
  python3 -c "import json;t=json.load(open('$O/traffic_$cfg.json'));print('$cfg', round(t['bytes_per_token'],1),'B/tok', {k:round(v,1) for k,v in t.get('per_token',{}).items()}, 'clk', round(t.get('effective_clock_ghz',0),3))"
}
prof c4 "k_sample<8, 3, false>" 250000000 512 && \
prof c2 "k_sample<2, 4, false>" 20000000 128 && \
prof c3 "k_sample<16, 2, false>" 20000000 1024 && \
prof c5 "k_sample_sparse_big<64, 4, false>" 250000000 4096 || exit 1
for cfg in c4 c2 c3 c5; do
  extra="--no-cpu-baseline"; [ $cfg = c4 ] && extra=""
  timeout -k 10 600 python bench.py --config $cfg $extra > $O/bench_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log > $O/bench_$cfg.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$cfg.jsonl').read());r=d['roofline'];i=r.get('issue') or {};print('$cfg', round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],3),'traffic_frac',r['traffic_frac'],'issue',i.get('binding'),i.get('frac'))"
done
timeout -k 10 600 python tools/opt_cost.py > $O/opt_cost.json 2> $O/opt_cost.log || { echo OPT_COST FAILED; tail -5 $O/opt_cost.log; exit 1; }
cat $O/opt_cost.json
