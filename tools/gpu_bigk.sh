set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "large_k or padding" > gpurun_out/pytest_bigk.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_bigk.log; exit 1; }
echo "pytest ok"; tail -2 gpurun_out/pytest_bigk.log
timeout -k 10 900 python bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || { echo BENCH c5 FAILED; tail -20 gpurun_out/bench_c5.log; exit 1; }
tail -1 gpurun_out/bench_c5.log
