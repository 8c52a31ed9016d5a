# Round 6, GPU call L: the after-burn-in windows of the dense samplers on
# this round's machine code -- C4 (whole corpus) and C2 after 30 sweeps:
# profile passes (tools/profile.sh, BURNIN=30), then the lines they match.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6l; mkdir -p $O
BURNIN=30 LABEL=r6_c4_b30 PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
BURNIN=30 LABEL=r6_c2_b30 BENCH_ARGS="--config c2" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
