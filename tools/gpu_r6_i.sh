# Round 6, GPU call I: the four-cells-per-word exchange (lda_set_exchange_cells)
# -- its exchange and distributed GPU tests, then the escapes per rank at 8
# ranks' biases on the C5 and C4 shards (tools/escape_rate.py) -- and call
# H's branch-free-rounds A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6i; mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_exchange_gpu.py tests/test_distributed_gpu.py > $O/pytest_exchange.log 2>&1 || { tail -30 $O/pytest_exchange.log; exit 1; }
tail -1 $O/pytest_exchange.log
for w in c5 c4shard; do
  timeout -k 10 300 python -u tools/escape_rate.py $w 8 > $O/escape_rate_$w.jsonl 2> $O/escape_rate_$w.err || { tail -20 $O/escape_rate_$w.err; exit 1; }
  cat $O/escape_rate_$w.jsonl
done
bash tools/gpu_r6_h.sh || exit 1
