set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5cnt; mkdir -p $O
LDA_MI355X_LIB=variants/xcount/liblda_mi355x.so timeout -k 10 600 python tools/count_paths.py 300000 0 5 30 > $O/count.log 2>&1 || { tail -20 $O/count.log; exit 1; }
cat $O/count.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu "tests/test_topic_model_gpu.py::test_staleness_sweeps_bit_exact" > $O/stale.log 2>&1; tail -2 $O/stale.log
