# Rehearse bench.py's N>1 path on one GPU: 4 ranks over gloo, small shards.
# (RCCL refuses two ranks on one device: "Duplicate GPU detected"; the nccl
# backend runs only on the driver's multi-GPU node.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 4 --warmup 1 --docs 50000 --backend gloo --no-cpu-baseline > gpurun_out/bench_4ranks_gloo.log 2>&1 || { echo "4-rank gloo bench FAILED"; tail -30 gpurun_out/bench_4ranks_gloo.log; exit 1; }
grep '"metric"' gpurun_out/bench_4ranks_gloo.log | cut -c1-400
