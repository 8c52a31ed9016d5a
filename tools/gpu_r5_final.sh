# Round 5's pending GPU work in one call, each step
# under its own time limit, stopping at the first failure:
#  1. the A searches from LDS (variants/apick, built with -DSB_APICK_LDS=1):
#     large-K parity on it, then C5 near init / after burn-in against the tree
#  2. the staleness test in both count modes
#  3. the whole GPU suite on the tree's library
#  4. C5 profile passes (traffic after burn-in) and the default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5f; mkdir -p $O
LDA_MI355X_LIB=variants/apick/liblda_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_parity_gpu.py -k "large_k or sparse" > $O/apick_parity.log 2>&1 \
  || { tail -20 $O/apick_parity.log; exit 1; }
tail -1 $O/apick_parity.log
bash tools/gpu_r5_c5ab.sh r5f 0 tree variants/apick/liblda_mi355x.so || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  "tests/test_topic_model_gpu.py::test_staleness_sweeps_bit_exact" > $O/stale.log 2>&1 || { tail -20 $O/stale.log; exit 1; }
tail -1 $O/stale.log
timeout -k 10 1000 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
  || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
