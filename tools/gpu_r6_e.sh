# Round 6, GPU call E: the final tree as the driver runs it -- every GPU test,
# smoke() -- then the lines carrying their round-6 traffic records (C5 near
# init and after 30 sweeps, C3, C2) and a 4-rank rehearsal of the default
# bench over gloo on one GPU (replicas, drop-in line).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6e; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for a in "c5 0" "c5 30" "c3 0" "c2 0"; do
  set -- $a
  timeout -k 10 400 python bench.py --config $1 --burnin $2 --no-cpu-baseline --no-estimate > $O/bench_$1_b$2.log 2>&1 || { tail -10 $O/bench_$1_b$2.log; exit 1; }
  tail -n 1 $O/bench_$1_b$2.log > $O/bench_$1_b$2.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$1_b$2.jsonl').read());r=d['roofline'];print('$1 b$2', round(d['value']/1e9,4), 'frac', round(r['frac'],3), 'traffic', r['traffic'] is not None, 'issue', (r['issue'] or {}).get('frac'), 'src', r['traffic_source'])"
done
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29543 \
  bench.py --gpus 4 --steps 3 --warmup 1 --docs 12500 --backend gloo --no-cpu-baseline > $O/bench_4ranks.log 2>&1 \
  || { tail -30 $O/bench_4ranks.log; exit 1; }
grep '^{' $O/bench_4ranks.log | tail -1 > $O/bench_4ranks.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_4ranks.jsonl').read());c=d['collective'];print('4 ranks', round(d['value']/1e9,3), c['replicas_agree'], c['ranks_counted'], d['dropin_schedule']['exchanges_per_sweep'])"
