# bench.py's N > 1 path on one GPU over gloo, with stack dumps every 40 s.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
LDA_BENCH_STACKS=40 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NR:-2} --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus ${NR:-2} --steps 2 --warmup 1 --docs ${DOCS:-20000} --backend gloo --no-cpu-baseline > gpurun_out/bench_ranks${NR:-2}_dbg.log 2>&1
rc=$?
grep '"metric"' gpurun_out/bench_ranks${NR:-2}_dbg.log | cut -c1-300
exit $rc
