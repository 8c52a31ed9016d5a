# Round evidence for the library in the tree: every -m gpu test, smoke, rocprofv3
# kernel trace + PMC passes on the C4 bench command, the PMC traffic file for
# THIS library, then the bench lines (C4 default with cpu_baseline and traffic;
# C1, C2, C3, C5).  Everything lands in gpurun_out/final/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
echo "pytest: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
PASSES="kt fetch write tcc sq lds" LABEL=final_c4 bash tools/profile.sh > $O/profile.log 2>&1 || { echo PROFILE FAILED; tail -20 $O/profile.log; exit 1; }
cp gpurun_out/prof_final_c4/summary_*.json gpurun_out/prof_final_c4/*kernel_stats.csv $O/ 2>/dev/null
python3 tools/make_traffic.py gpurun_out/prof_final_c4 "k_sample<8, 3, false>" 250000000 c4 $O/traffic_k512.json || { echo TRAFFIC FAILED; exit 1; }
cp $O/traffic_k512.json profiles/r01/traffic_k512.json
for cfg in c4 c1 c2 c3 c5; do
  extra=""; [ $cfg != c4 ] && extra="--no-cpu-baseline"; [ $cfg = c1 ] && extra=""
  timeout -k 10 600 python bench.py --config $cfg $extra > $O/bench_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log > $O/bench_$cfg.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$cfg.jsonl').read());r=d['roofline'];print('$cfg', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms/step kernel',round(r['kernel_ms_timed_region'],3),'traffic',r['traffic'])"
done
# the C4 rate after 30 burn-in sweeps (counts concentrated; no traffic file for it)
timeout -k 10 600 python bench.py --config c4 --burnin 30 --no-cpu-baseline > $O/bench_c4_b30.log 2>&1 || { echo "BENCH c4 b30 FAILED"; tail -5 $O/bench_c4_b30.log; exit 1; }
tail -1 $O/bench_c4_b30.log > $O/bench_c4_b30.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_c4_b30.jsonl').read());print('c4 burnin 30', round(d['value']/1e9,4),'Gtok/s')"
