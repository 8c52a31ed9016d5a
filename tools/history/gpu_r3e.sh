# Round 3 evidence on the tree's library: bench lines (the default = whole C4,
# C2, C3, C5, C1) and rocprofv3 passes of the same bench commands (same
# warm-up / timed window: tools/profile.sh skips the warm-up dispatches), the
# traffic files bench.py reads (profiles/r03/traffic_<cfg>.json), then the
# bench lines again so they carry the PMC traffic.  Output: gpurun_out/r3e/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3e; mkdir -p $O profiles/r03
export TMPDIR=/tmp
prof() {  # label, kernel, tokens, K, bench args
  local L=$1 KN=$2 TOK=$3 K=$4; shift 4
  PASSES="kt fetch write sq lds grbm" LABEL=$L BENCH_ARGS="$*" bash tools/profile.sh > $O/profile_$L.log 2>&1 || { echo "PROFILE $L FAILED"; tail -20 $O/profile_$L.log; return 1; }
  mkdir -p $O/prof_$L && cp gpurun_out/prof_$L/summary_*.json $O/prof_$L/ && cp gpurun_out/prof_$L/*kernel_stats.csv $O/prof_$L/ 2>/dev/null
  python3 tools/make_traffic.py gpurun_out/prof_$L "$KN" $TOK "$L" $O/traffic_$L.json $K > /dev/null || { echo "TRAFFIC $L FAILED"; return 1; }
  cp $O/traffic_$L.json profiles/r03/traffic_$L.json
  echo "profile $L ok"
}
line() {  # name, bench args
  local N=$1; shift
  timeout -k 10 900 python bench.py "$@" > $O/bench_$N.log 2>&1 || { echo "BENCH $N FAILED"; tail -5 $O/bench_$N.log; return 1; }
  tail -1 $O/bench_$N.log > $O/bench_$N.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$N.jsonl').read());r=d['roofline'];print('$N', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms kernel',round(r['kernel_ms_timed_region'],3),'frac',round(r['frac'],3),'traffic',r.get('traffic'),'traffic_frac',r.get('traffic_frac'))"
}
# two calls (each under gpurun's 20-minute limit): "prof" then "lines"
# ("profc4c2": the C4 and C2 profiles alone, after a large-K-only change)
case ${1:-all} in
  prof|all) prof c4 "k_sample<8, 3, false>" 2000000000 512 --config c4 && \
            prof c2 "k_sample_quarter<8, 4, false>" 20000000 128 --config c2 && \
            prof c5 "k_sample_sparse_big<64, 3, false>" 250000000 4096 --config c5 || exit 1 ;;
esac
case ${1:-all} in
  profc4c2) prof c4 "k_sample<8, 3, false>" 2000000000 512 --config c4 && \
            prof c2 "k_sample_quarter<8, 4, false>" 20000000 128 --config c2 || exit 1 ;;
esac
case ${1:-all} in
  lines|all) line c4 && line c2 --config c2 --no-cpu-baseline && line c3 --config c3 --no-cpu-baseline && \
             line c5 --config c5 --no-cpu-baseline && line c1 --config c1 --no-cpu-baseline && \
             line c4shard --config c4shard --no-cpu-baseline || exit 1 ;;
esac
