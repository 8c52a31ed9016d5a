# Round 6, GPU call J: the exchange tests again with ADLDATrainer's
# four-cells default for large K (one-rank RCCL at K = 2048), a 2-rank gloo
# rehearsal of the C5 bench on one GPU (four cells per word, replicas), then
# call H's branch-free-rounds A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6j; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_exchange_gpu.py tests/test_distributed_gpu.py > $O/pytest_exchange.log 2>&1 || { tail -30 $O/pytest_exchange.log; exit 1; }
tail -1 $O/pytest_exchange.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29547 \
  bench.py --gpus 2 --config c5 --steps 3 --warmup 1 --docs 100000 --backend gloo --no-cpu-baseline > $O/bench_2ranks_c5.log 2>&1 \
  || { tail -30 $O/bench_2ranks_c5.log; exit 1; }
grep '^{' $O/bench_2ranks_c5.log | tail -1 > $O/bench_2ranks_c5.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_2ranks_c5.jsonl').read());c=d['collective'];print('2 ranks c5', round(d['value']/1e9,3), c['replicas_agree'], c['cells_per_word'], c['escape_count_max'], c['allreduce_bytes_per_part'], d['dropin_schedule'].get('exchanges_per_sweep'))"
bash tools/gpu_r6_h.sh || exit 1
