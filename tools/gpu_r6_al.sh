# Round 6, GPU call AL: the final library as the driver runs it -- smoke(),
# the default line (python bench.py), then the C3 and C2 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6al; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
s=$(date +%s)
timeout -k 10 900 python bench.py > $O/bench_default.log 2>&1 || { tail -10 $O/bench_default.log; exit 1; }
echo "bench wall $(( $(date +%s) - s )) s"
tail -n 1 $O/bench_default.log > $O/bench_c4_default.jsonl
for c in c3 c2; do
  timeout -k 10 600 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -10 $O/bench_$c.log; exit 1; }
  tail -n 1 $O/bench_$c.log > $O/bench_$c.jsonl
done
for f in $O/bench_c4_default.jsonl $O/bench_c3.jsonl $O/bench_c2.jsonl; do
  python3 -c "import json;d=json.loads(open('$f').read());r=d['roofline'];print('$f'.split('/')[-1], round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],4),'traffic',r.get('traffic') is not None,'issue',(r.get('issue') or {}).get('frac'))"
done
