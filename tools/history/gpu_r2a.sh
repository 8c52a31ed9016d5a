# Round-2 step A: the new config-scale / >2^31 / race / inference tests, then
# the whole -m gpu suite and smoke (each step under its own time limit).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r2a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_configs_gpu.py tests/test_distributed_gpu.py \
  "tests/test_parity_gpu.py::test_dense_16bit_row_boundary" \
  "tests/test_parity_gpu.py::test_inference_skips_types_without_training_tokens" \
  -x -v --timeout 400 --timeout-method thread --durations=0 > $O/pytest_new.log 2>&1 \
  || { echo "NEW TESTS FAILED"; tail -60 $O/pytest_new.log; exit 1; }
echo "new: $(tail -1 $O/pytest_new.log)"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread --durations=15 > $O/pytest_gpu.log 2>&1 \
  || { echo "SUITE FAILED"; tail -40 $O/pytest_gpu.log; exit 1; }
echo "suite: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
