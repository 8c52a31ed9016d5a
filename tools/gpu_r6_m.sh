# Round 6, GPU call M: the native ShardGroup's used-length escape lists and
# four-cell exchange for large K (LDA_LOCAL_COMPACT stand-ins on one GPU),
# then the topic-model, JNI-harness and exchange GPU tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_topic_model_gpu.py tests/test_jni_harness_gpu.py tests/test_exchange_gpu.py > $O/pytest.log 2>&1
rc=$?; tail -n 5 $O/pytest.log; exit $rc
