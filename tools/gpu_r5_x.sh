set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_exchange_gpu.py tests/test_distributed_gpu.py "tests/test_parity_gpu.py::test_large_k_ring_probe_with_empty_first_part" "tests/test_topic_model_gpu.py::test_shard_group_compact_exchange_on_one_device" "tests/test_topic_model_gpu.py::test_shard_group_on_one_device" > $O/xch.log 2>&1; rc=$?; tail -4 $O/xch.log; [ $rc -eq 0 ] || exit 1
# N=2 rehearsal on one GPU (gloo; rates not meaningful) + one-rank RCCL forced exchange: the replica fields
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 4 --warmup 1 --docs 50000 --backend gloo --no-cpu-baseline > $O/bench_2ranks.log 2>&1 || { tail -20 $O/bench_2ranks.log; exit 1; }
grep '^{' $O/bench_2ranks.log > $O/bench_2ranks.jsonl
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29542 bench.py --gpus 2 --steps 3 --warmup 1 --config c5 --docs 60000 --backend gloo --no-cpu-baseline > $O/bench_2ranks_c5.log 2>&1 || { tail -20 $O/bench_2ranks_c5.log; exit 1; }
grep '^{' $O/bench_2ranks_c5.log > $O/bench_2ranks_c5.jsonl
timeout -k 10 600 python bench.py --force-exchange --steps 5 --warmup 1 --no-cpu-baseline --no-estimate > $O/c4_force.jsonl 2> $O/c4_force.err || { tail -20 $O/c4_force.err; exit 1; }
python3 -c "
import json
for f in ['bench_2ranks.jsonl','bench_2ranks_c5.jsonl','c4_force.jsonl']:
    d=json.loads(open('$O/'+f).read().strip().splitlines()[-1]); c=d['collective']
    print(f, d['n_gpus'], c['replicas_agree'], c['world_size'], c['ranks_counted'], c['rank_ms_per_sweep'], c['escape_lists'], c['escape_count_max'], c['allgather_bytes_per_part'], c['allgather_capacity_bytes_per_part'])
"
