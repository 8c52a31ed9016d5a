# Round 3, step AI: profiles of the after-burn-in windows (the bench command
# with --burnin 30: the summaries skip the burn-in and warm-up dispatches) for
# C5 and the whole-C4 default, their traffic files (with "burnin": 30, which
# bench.py matches), then the after-30-sweeps lines that now carry their own
# window's traffic.  Output: gpurun_out/r3ai/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ai; mkdir -p $O profiles/r03
export TMPDIR=/tmp
prof() {  # label, kernel, tokens, K, bench args
  local L=$1 KN=$2 TOK=$3 K=$4; shift 4
  BURNIN=30 PASSES="kt fetch write sq lds grbm" LABEL=$L BENCH_ARGS="$*" bash tools/profile.sh > $O/profile_$L.log 2>&1 || { echo "PROFILE $L FAILED"; tail -20 $O/profile_$L.log; return 1; }
  mkdir -p $O/prof_$L && cp gpurun_out/prof_$L/summary_*.json $O/prof_$L/ && cp gpurun_out/prof_$L/*kernel_stats.csv $O/prof_$L/ 2>/dev/null
  python3 tools/make_traffic.py gpurun_out/prof_$L "$KN" $TOK "$L" $O/traffic_$L.json $K 30 > /dev/null || { echo "TRAFFIC $L FAILED"; return 1; }
  cp $O/traffic_$L.json profiles/r03/traffic_$L.json
  echo "profile $L ok"
}
line() {  # name, bench args
  local N=$1; shift
  timeout -k 10 900 python bench.py "$@" > $O/bench_$N.log 2>&1 || { echo "BENCH $N FAILED"; tail -5 $O/bench_$N.log; return 1; }
  tail -1 $O/bench_$N.log > $O/bench_$N.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$N.jsonl').read());r=d['roofline'];print('$N', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms kernel',round(r['kernel_ms_timed_region'],3),'frac',round(r['frac'],3),'traffic',r.get('traffic'),'traffic_frac',r.get('traffic_frac'),r.get('traffic_source'))"
}
prof c5_b30 "k_sample_sparse_big<64, 3, false>" 250000000 4096 --config c5 && \
prof c4_b30 "k_sample<8, 3, false>" 2000000000 512 --config c4 && \
line c5_b30 --config c5 --burnin 30 --no-cpu-baseline && line c4_b30 --burnin 30 --no-cpu-baseline || exit 1
