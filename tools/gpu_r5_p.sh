# C5 after 30 burn-in sweeps: tree (kt fetch write sq lds sq2) and the
# no-doc-part attribution variant (sq lds sq2), fixed default ring
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export LDA_SB_RB=default
bash tools/gpu_r5_prof.sh r5p_tree 30 "kt fetch write sq lds sq2" --config c5 || exit 1
LDA_MI355X_LIB=variants/xnoa/liblda_mi355x.so bash tools/gpu_r5_prof.sh r5p_xnoa 30 "kt sq lds sq2" --config c5 || exit 1
