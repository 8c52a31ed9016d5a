# Round 3, step X: the statistics kernels with block-level aggregation (doc
# histogram) and fewer blocks (count histogram): the statistics / optimisation
# tests, then the reference runs and the estimate() overhead split.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3x; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_hyper_gpu.py tests/test_topic_model_gpu.py \
  tests/test_jni_harness_gpu.py > $O/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "FAILED|Error" $O/tests.log | head; tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs.log 2>&1 || { echo "REFRUNS FAILED"; tail -5 $O/reference_runs.log; exit 1; }
grep -E "^src/" $O/reference_runs.log
timeout -k 10 300 python tools/estimate_overhead.py > $O/est_overhead.json 2> $O/est_overhead.err || { echo "OVERHEAD FAILED"; tail -5 $O/est_overhead.err; exit 1; }
cat $O/est_overhead.json
