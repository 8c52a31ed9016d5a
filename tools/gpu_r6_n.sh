# Round 6, GPU call N: parity over 96 (then 256) randomly drawn configurations
# (tests/test_parity_random_gpu.py: every kernel family, schedules, count
# modes, split sweeps, token bases above 2^32, inference).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 120 --timeout-method thread -m gpu \
  tests/test_parity_random_gpu.py > $O/pytest_random.log 2>&1
rc=$?; tail -n 30 $O/pytest_random.log; exit $rc
