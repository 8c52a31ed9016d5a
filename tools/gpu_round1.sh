set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocminfo 2>/dev/null | grep -m2 -E "Marketing|gfx" > gpurun_out/device.txt || true
nproc > gpurun_out/nproc.txt; lscpu | head -20 >> gpurun_out/nproc.txt
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest ok"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE FAILED; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --docs 100000 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 || { echo BENCH SMALL FAILED; tail -30 gpurun_out/bench_small.log; exit 1; }
cat gpurun_out/bench_small.log
timeout -k 10 900 python bench.py > gpurun_out/bench_full.log 2>&1 || { echo BENCH FULL FAILED; tail -30 gpurun_out/bench_full.log; exit 1; }
cat gpurun_out/bench_full.log
