# Round-2 step C: FETCH/WRITE calibration on known bytes, then the PMC passes
# of the v6 large-K sampler on the C5 bench command.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_calib.sh || exit 1
PASSES="kt fetch write sq lds grbm" LABEL=c5 BENCH_ARGS="--config c5" bash tools/profile.sh > gpurun_out/profile_c5.log 2>&1 || { echo "PROFILE c5 FAILED"; tail -20 gpurun_out/profile_c5.log; exit 1; }
echo "profile c5 ok"
