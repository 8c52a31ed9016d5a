# Round 3, step Q: the final library as the driver runs it -- every GPU test,
# smoke(), the default bench line -- plus a 2-rank rehearsal of the default
# (whole-C4-split) bench path on one GPU over gloo (blocking and split
# exchange; 25k documents per block), since the 8-GPU node is the driver's.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3q; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for ex in 1 2; do
  timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 2954$ex \
    bench.py --gpus 2 --steps 4 --warmup 1 --docs 25000 --backend gloo --exchange-parts $ex --no-cpu-baseline \
    > $O/bench_2ranks_parts$ex.log 2>&1 || { echo "2-rank bench parts $ex FAILED"; tail -30 $O/bench_2ranks_parts$ex.log; exit 1; }
  grep '^{' $O/bench_2ranks_parts$ex.log | tail -1 > $O/bench_2ranks_parts$ex.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_2ranks_parts$ex.jsonl').read());print('2 ranks parts $ex', d['n_gpus'], round(d['value']/1e9,3), 'Gtok/s', d['config']['tokens_all_gpus'], 'tokens', d.get('collective'))"
done
timeout -k 10 900 python bench.py > $O/bench.log 2>&1 || { echo "BENCH FAILED"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.jsonl
python3 -c "import json;d=json.loads(open('$O/bench.jsonl').read());r=d['roofline'];print('default', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],3),'ms frac',round(r['frac'],3),'traffic_frac',r.get('traffic_frac'))"
