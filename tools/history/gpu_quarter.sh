# Quarter-wave dense sampler (K <= 128, LDA_DENSE_HALF=2): its parity tests,
# then C2 bench lines for the default k_sample<2>, the half-wave and the
# quarter-wave variant (same library, selected by the environment).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/quarter
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k half_wave -x -v --timeout 120 --timeout-method thread > gpurun_out/quarter/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 gpurun_out/quarter/parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/quarter/parity.log)"
for v in 0 1 2; do
  for b in 0 30; do
    LDA_DENSE_HALF=$v timeout -k 10 240 python -u bench.py --config c2 --steps 20 --warmup 3 --burnin $b --no-cpu-baseline > gpurun_out/quarter/bench_v${v}_b${b}.json 2> gpurun_out/quarter/bench_v${v}_b${b}.err || { echo "BENCH v$v b$b FAILED"; tail -20 gpurun_out/quarter/bench_v${v}_b${b}.err; exit 1; }
    echo "v$v burnin$b: $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/quarter/bench_v${v}_b${b}.json)"
  done
done
