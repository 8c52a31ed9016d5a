# SQ / LDS instruction counters of the large-K sparse kernel on the C5 shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
PASSES="sq lds" LABEL=c5 BENCH_ARGS="--config c5" bash tools/profile.sh
