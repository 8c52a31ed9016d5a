set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_bench_ranks.sh || exit 1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 4 --warmup 1 --docs 50000 --backend gloo --exchange-parts 3 --no-cpu-baseline > gpurun_out/bench_2ranks_gloo_split.log 2>&1 || { echo "split FAILED"; tail -30 gpurun_out/bench_2ranks_gloo_split.log; exit 1; }
grep '"metric"' gpurun_out/bench_2ranks_gloo_split.log | cut -c1-300
