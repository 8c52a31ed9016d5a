# Round 6: GPU calls F then E in one lease (tools/gpu_r6_f.sh, tools/gpu_r6_e.sh)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r6_f.sh || exit 1
bash tools/gpu_r6_e.sh || exit 1
