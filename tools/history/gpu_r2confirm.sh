# Confirmation on the libraries rebuilt from the committed sources: every -m gpu
# test, smoke, the default bench line and C2 (quarter-wave) at burn-in 0 / 30.
# Everything under gpurun_out/confirm/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/confirm; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=10 > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -60 $O/pytest_gpu.log; exit 1; }
echo "pytest: $(grep -E 'passed|failed' $O/pytest_gpu.log | tail -1)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { echo "BENCH FAILED"; tail -5 $O/bench_default.log; exit 1; }
tail -1 $O/bench_default.log > $O/bench_default.jsonl
for b in 0 30; do
  timeout -k 10 300 python bench.py --config c2 --burnin $b --no-cpu-baseline > $O/bench_c2_b$b.log 2>&1 || { echo "BENCH c2 b$b FAILED"; tail -5 $O/bench_c2_b$b.log; exit 1; }
  tail -1 $O/bench_c2_b$b.log > $O/bench_c2_b$b.jsonl
done
for f in $O/bench_*.jsonl; do
  python3 -c "import json;d=json.loads(open('$f').read());r=d['roofline'];print('$f', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms frac',round(r['frac'],3), r.get('kernel'))"
done
