# Round 6, GPU call AN: the final large-K sampler (document counts from the chunk registers, the ring
# refilled first, the early batch, ...) -- every GPU test, smoke(), the C5 profiles near
# init and after 30 sweeps, their traffic records (written into the box's
# profiles/ so the lines below find them, and copied to gpurun_out/), then the
# C5 lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6an; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
LABEL=r6_c5d BENCH_ARGS="--config c5" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
BURNIN=30 LABEL=r6_c5d_b30 BENCH_ARGS="--config c5" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh >> $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/make_traffic.py gpurun_out/prof_r6_c5d "k_sample_big<64, 2, 12, false>" 250000000 \
  "c5 shard near init (round 6, batched LDS reads, global atomics, prefixes in registers, sparse doc part, early long-row batch, refill first, doc counts from registers)" profiles/r06/traffic_c5_final.json 4096 > $O/traffic.log 2>&1 || { tail $O/traffic.log; exit 1; }
python3 tools/make_traffic.py gpurun_out/prof_r6_c5d_b30 "k_sample_big<64, 4, 6, false>" 250000000 \
  "c5 shard after 30 burn-in sweeps (round 6, batched LDS reads, global atomics, prefixes in registers, sparse doc part, early long-row batch, refill first, doc counts from registers; the timed ring)" profiles/r06/traffic_c5_final_b30.json 4096 30 >> $O/traffic.log 2>&1 || { tail $O/traffic.log; exit 1; }
cp profiles/r06/traffic_c5_final.json profiles/r06/traffic_c5_final_b30.json $O/
for bi in 0 30; do
  timeout -k 10 600 python bench.py --config c5 --burnin $bi > $O/bench_c5_b$bi.log 2>&1 || { tail -10 $O/bench_c5_b$bi.log; exit 1; }
  tail -n 1 $O/bench_c5_b$bi.log > $O/bench_c5_b$bi.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_c5_b$bi.jsonl').read());r=d['roofline'];print('c5 b$bi', round(d['value']/1e9,4),'Gtok/s frac',round(r['frac'],4),'traffic',r.get('traffic'),'src',r.get('traffic_source'),'issue',(r.get('issue') or {}).get('frac'))"
done
