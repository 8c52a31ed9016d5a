# Round evidence: GPU tests, default bench line, rocprof summaries + PMC traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
LABEL=${LABEL:-evidence}
timeout -k 10 1200 python -m pytest tests -m gpu -q -k "not perplexity" > gpurun_out/pytest_gpu_$LABEL.log 2>&1 || { echo "PYTEST FAILED rc=$?"; tail -60 gpurun_out/pytest_gpu_$LABEL.log; exit 1; }
echo "pytest ok"; tail -2 gpurun_out/pytest_gpu_$LABEL.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$LABEL.log 2>&1 || { echo BENCH FAILED; tail -20 gpurun_out/bench_$LABEL.log; exit 1; }
tail -1 gpurun_out/bench_$LABEL.log
PASSES="kt fetch write tcc" LABEL=$LABEL bash tools/profile.sh || exit 1
python3 tools/make_traffic.py gpurun_out/prof_$LABEL "k_sample<8, 2, false>" 250000000 c4 gpurun_out/prof_$LABEL/traffic_k512.json
