# Round 3, step AE: evidence on the v8.4 library -- every GPU test, smoke(),
# the C5 profile of the bench command itself (kernel trace + PMC passes, the
# traffic file bench.py reads), the C5 lines near init and after 30 sweeps,
# and the default (whole-C4) line.  Output: gpurun_out/r3ae/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ae; mkdir -p $O profiles/r03
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
L=c5; KN="k_sample_sparse_big<64, 3, false>"
PASSES="kt fetch write sq lds grbm" LABEL=$L BENCH_ARGS="--config c5" bash tools/profile.sh > $O/profile_$L.log 2>&1 || { echo "PROFILE $L FAILED"; tail -20 $O/profile_$L.log; exit 1; }
mkdir -p $O/prof_$L && cp gpurun_out/prof_$L/summary_*.json $O/prof_$L/ && cp gpurun_out/prof_$L/*kernel_stats.csv $O/prof_$L/ 2>/dev/null
python3 tools/make_traffic.py gpurun_out/prof_$L "$KN" 250000000 "$L" $O/traffic_$L.json 4096 > /dev/null || { echo "TRAFFIC $L FAILED"; exit 1; }
cp $O/traffic_$L.json profiles/r03/traffic_$L.json
echo "profile $L ok"
line() {  # name, bench args
  local N=$1; shift
  timeout -k 10 900 python bench.py "$@" > $O/bench_$N.log 2>&1 || { echo "BENCH $N FAILED"; tail -5 $O/bench_$N.log; return 1; }
  tail -1 $O/bench_$N.log > $O/bench_$N.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$N.jsonl').read());r=d['roofline'];print('$N', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms kernel',round(r['kernel_ms_timed_region'],3),'frac',round(r['frac'],3),'traffic',r.get('traffic'),'traffic_frac',r.get('traffic_frac'))"
}
line c5 --config c5 --no-cpu-baseline && line c5_b30 --config c5 --burnin 30 --no-cpu-baseline && line default || exit 1
