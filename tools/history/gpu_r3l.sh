# Round 3, step L: the round's library as the driver runs it: every GPU test,
# smoke(), the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -10 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.jsonl
python3 -c "import json;d=json.loads(open('$O/bench.jsonl').read());r=d['roofline'];print(round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms frac',round(r['frac'],3), 'recount', r['count_update'], r['recount_ms_timed_region'])"
