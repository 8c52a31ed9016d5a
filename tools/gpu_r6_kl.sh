# Round 6: GPU calls K and L in one lease (the final suite, the after-burn-in
# profiles, the reference's own scale)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/gpu_r6_l.sh || exit 1
for cfg in c1 c1cmu c1ron; do
  timeout -k 10 300 python bench.py --config $cfg > $O/bench_$cfg.log 2>&1 || { tail -10 $O/bench_$cfg.log; exit 1; }
  tail -n 1 $O/bench_$cfg.log > $O/bench_$cfg.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$cfg.jsonl').read());print('$cfg', round(d['value']/1e6,1), 'Mtok/s', round(d['ms_per_step']*1e3,1), 'us/sweep; cpu', round(d['cpu_baseline']['value']/1e6,2))"
done
timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs.log 2>&1 || { tail -20 $O/reference_runs.log; exit 1; }
tail -6 $O/reference_runs.log
