# Round 6, GPU call T: the tree with the batched LDS reads -- every GPU test,
# smoke(), then the C5 lines near init and after 30 sweeps carrying their new
# traffic records.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for bi in 0 30; do
  timeout -k 10 600 python bench.py --config c5 --burnin $bi > $O/bench_c5_b$bi.log 2>&1 || { tail -10 $O/bench_c5_b$bi.log; exit 1; }
  tail -n 1 $O/bench_c5_b$bi.log > $O/bench_c5_b$bi.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_c5_b$bi.jsonl').read());r=d['roofline'];print('c5 b$bi', round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],4),'traffic',r.get('traffic'),'src',r.get('traffic_source'),'issue',(r.get('issue') or {}).get('frac'))"
done
