set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python tools/reference_runs.py > gpurun_out/reference_runs.log 2>&1 || { echo FAILED; tail -20 gpurun_out/reference_runs.log; exit 1; }
grep -v amdgpu.ids gpurun_out/reference_runs.log
timeout -k 10 300 python bench.py --config c1 > gpurun_out/bench_c1.log 2>&1 || { echo C1 FAILED; tail -20 gpurun_out/bench_c1.log; exit 1; }
tail -1 gpurun_out/bench_c1.log
