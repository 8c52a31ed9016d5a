set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "large_k or padding" > gpurun_out/pytest_bigk.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_bigk.log; exit 1; }
echo "pytest ok"; tail -2 gpurun_out/pytest_bigk.log
timeout -k 10 900 python bench.py --config c5 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_c5.log 2>&1 || { echo BENCH c5 FAILED; tail -20 gpurun_out/bench_c5.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_c5.log').read().strip().splitlines()[-1]);print('c5', round(d['value']/1e9,4), 'Gtok/s', d['ms_per_step'], d['roofline']['kernel'], d['ll_per_token'])"
timeout -k 10 900 python bench.py --config c5 --burnin 30 --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bench_c5_b30.log 2>&1 || { echo BENCH c5 b30 FAILED; tail -20 gpurun_out/bench_c5_b30.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_c5_b30.log').read().strip().splitlines()[-1]);print('c5 b30', round(d['value']/1e9,4), 'Gtok/s', d['ms_per_step'], d['roofline']['kernel'], d['ll_per_token'])"
