set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_topic_model_gpu.py -m gpu -q -x > gpurun_out/pytest_dense.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_dense.log; exit 1; }
echo "pytest ok"; tail -2 gpurun_out/pytest_dense.log
for cfg in c4 c2 c3; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_dense_$cfg.log 2>&1 || { echo BENCH $cfg FAILED; tail -20 gpurun_out/bench_dense_$cfg.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_dense_$cfg.log').read().strip().splitlines()[-1]);print('$cfg', round(d['value']/1e9,4), 'Gtok/s', d['roofline']['kernel'])"
done
