set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python tools/small_corpus.py 0 1 16 64 256 > gpurun_out/small_corpus.log 2>&1 || { echo FAILED; tail -20 gpurun_out/small_corpus.log; exit 1; }
cat gpurun_out/small_corpus.log
