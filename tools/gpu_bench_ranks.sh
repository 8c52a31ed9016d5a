# Rehearse bench.py's N>1 path on one GPU: 2 ranks, gloo, small shards.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 4 --warmup 1 --docs 50000 --backend gloo --no-cpu-baseline > gpurun_out/bench_2ranks.log 2>&1 || { echo "2-rank bench FAILED"; tail -30 gpurun_out/bench_2ranks.log; exit 1; }
grep '"metric"' gpurun_out/bench_2ranks.log
