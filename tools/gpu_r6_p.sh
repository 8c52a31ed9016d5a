# Round 6, GPU call P: the final tree as the driver runs it -- every GPU test,
# smoke(), the default bench line (python bench.py, timed end to end).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6p; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
s=$(date +%s)
timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1 || { tail -10 $O/bench_default.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
tail -n 1 $O/bench_default.log > $O/bench_c4_default.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_c4_default.jsonl').read());r=d['roofline'];print(round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],4),'traffic',r.get('traffic'),'cpu',d['cpu_baseline']['value'], 'dropin', (d.get('dropin_schedule') or {}).get('value'))"
