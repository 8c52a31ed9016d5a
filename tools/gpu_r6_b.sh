# Round 6, GPU call B: profiles on the shipped sources (SB_APICK_LDS on) --
# C5 near init and after 30 burn-in sweeps, C3 -- each pass its own rocprofv3
# run (tools/profile.sh), then the lines they are matched to.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b; mkdir -p $O
LABEL=r6_c5 BENCH_ARGS="--config c5" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
BURNIN=30 LABEL=r6_c5_b30 BENCH_ARGS="--config c5" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
LABEL=r6_c3 BENCH_ARGS="--config c3" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
