set -o pipefail
cd "$GRAFT_REPO_ROOT"
PASSES="kt sq lds" LABEL=c2half BENCH_ARGS="--config c2" bash tools/profile.sh > gpurun_out/profile_c2half.log 2>&1 || { echo FAIL1; tail gpurun_out/profile_c2half.log; exit 1; }
LDA_MI355X_LIB=$PWD/variants/fullwave/liblda_mi355x.so PASSES="kt sq lds" LABEL=c2full BENCH_ARGS="--config c2" bash tools/profile.sh > gpurun_out/profile_c2full.log 2>&1 || { echo FAIL2; tail gpurun_out/profile_c2full.log; exit 1; }
echo ok
