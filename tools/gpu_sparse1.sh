set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 1200 python -m pytest tests -m gpu -x -q -k "not perplexity" > gpurun_out/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
echo "pytest ok"; tail -2 gpurun_out/pytest_gpu.log
for smp in dense sparse; do
  timeout -k 10 600 python bench.py --sampler $smp --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_$smp.log 2>&1 || { echo BENCH $smp FAILED; tail -20 gpurun_out/bench_$smp.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/bench_$smp.log').read().strip().splitlines()[-1]);print('$smp', d['value']/1e9, 'Gtok/s', d['roofline']['kernel'])"
done
timeout -k 10 600 python bench.py --sampler sparse --burnin 50 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_sparse_b50.log 2>&1 || { echo BENCH sparse burnin FAILED; tail -20 gpurun_out/bench_sparse_b50.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_sparse_b50.log').read().strip().splitlines()[-1]);print('sparse burnin50', d['value']/1e9, 'Gtok/s', d['roofline']['kernel'], d['ll_per_token'])"
timeout -k 10 600 python bench.py --sampler dense --burnin 50 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_dense_b50.log 2>&1 || { echo BENCH dense burnin FAILED; tail -20 gpurun_out/bench_dense_b50.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_dense_b50.log').read().strip().splitlines()[-1]);print('dense burnin50', d['value']/1e9, 'Gtok/s', d['roofline']['kernel'], d['ll_per_token'])"
