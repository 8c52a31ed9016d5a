# Round-2 final evidence for the library in the tree: every -m gpu test and
# smoke, PMC passes (kernel trace, FETCH, WRITE, SQ mix, LDS/SALU, GRBM) of the
# sampler at C4 / C2 / C3 / C5 with their traffic files, then the bench lines
# that read them, and the hyperparameter-optimisation cost at the C4 shard.
# Everything under gpurun_out/final/; traffic files also into profiles/r02/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final2; mkdir -p $O profiles/r02
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -60 $O/pytest_gpu.log; exit 1; }
echo "pytest: $(grep -E 'passed|failed' $O/pytest_gpu.log | tail -1)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
prof() {  # cfg kernel tokens K
  local cfg=$1 kern=$2 tok=$3 K=$4
  PASSES="kt fetch write sq lds grbm" LABEL=$cfg BENCH_ARGS="--config $cfg" bash tools/profile.sh > $O/profile_$cfg.log 2>&1 || { echo "PROFILE $cfg FAILED"; tail -20 $O/profile_$cfg.log; return 1; }
  mkdir -p $O/prof_$cfg && cp gpurun_out/prof_$cfg/summary_*.json $O/prof_$cfg/ && cp gpurun_out/prof_$cfg/*kernel_stats.csv $O/prof_$cfg/ 2>/dev/null
  python3 tools/make_traffic.py gpurun_out/prof_$cfg "$kern" $tok $cfg $O/traffic_$cfg.json $K > /dev/null || { echo "TRAFFIC $cfg FAILED"; return 1; }
  cp $O/traffic_$cfg.json profiles/r02/traffic_$cfg.json
  python3 -c "import json;t=json.load(open('$O/traffic_$cfg.json'));print('$cfg', round(t['bytes_per_token'],1),'B/tok', {k:round(v,1) for k,v in t.get('per_token',{}).items()}, 'clk', round(t.get('effective_clock_ghz',0),3))"
}
prof c4 "k_sample<8, 3, false>" 250000000 512 && \
prof c2 "k_sample_quarter<8, 4, false>" 20000000 128 && \
prof c3 "k_sample<16, 2, false>" 20000000 1024 && \
prof c5 "k_sample_sparse_big<64, 3, false>" 250000000 4096 || exit 1
for cfg in c4 c1 c2 c3 c5; do
  extra="--no-cpu-baseline"; [ $cfg = c4 ] && extra=""
  timeout -k 10 600 python bench.py --config $cfg $extra > $O/bench_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log > $O/bench_$cfg.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$cfg.jsonl').read());r=d['roofline'];i=r.get('issue') or {};print('$cfg', round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],3),'traffic_frac',r.get('traffic_frac'),'issue',i.get('binding'),i.get('frac'))"
done
timeout -k 10 120 python bench.py --config c5 --burnin 30 --no-cpu-baseline > $O/bench_c5_b30.log 2>&1 && tail -1 $O/bench_c5_b30.log > $O/bench_c5_b30.jsonl
timeout -k 10 120 python bench.py --config c4 --burnin 30 --no-cpu-baseline > $O/bench_c4_b30.log 2>&1 && tail -1 $O/bench_c4_b30.log > $O/bench_c4_b30.jsonl
# the whole C4 corpus (2e9 tokens, int64 offsets) in one context on one GPU
timeout -k 10 300 python bench.py --config c4full --no-cpu-baseline --steps 5 --warmup 2 > $O/bench_c4full.log 2>&1 && tail -1 $O/bench_c4full.log > $O/bench_c4full.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_c4full.jsonl').read());print('c4full', round(d['value']/1e9,4),'Gtok/s', d['ms_per_step'],'ms/step')"
timeout -k 10 600 python tools/opt_cost.py > $O/opt_cost.json 2> $O/opt_cost.log || { echo OPT_COST FAILED; tail -5 $O/opt_cost.log; exit 1; }
cat $O/opt_cost.json
