# rocprofv3 passes of one C5 bench command for the tree's library (or
# LDA_MI355X_LIB), per-token instruction mix printed.
#   bash tools/gpu_r5_prof.sh OUT BURNIN PASSES [bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$1; BI=$2; PS=$3; shift 3
BURNIN=$BI PASSES="$PS" LABEL=$O BENCH_ARGS="$*" bash tools/profile.sh > gpurun_out/profile_$O.log 2>&1 || { echo "PROFILE FAILED"; tail -20 gpurun_out/profile_$O.log; exit 1; }
python3 - "$O" <<'PY'
import json, os, sys
d = "gpurun_out/prof_" + sys.argv[1]
for f in sorted(os.listdir(d)):
    if not f.startswith("summary_"): continue
    j = json.load(open(os.path.join(d, f)))
    for k, v in j.get("counters", {}).items():
        if "sample" in k:
            print(f, k[:60], {c: round(x["avg_per_dispatch"] / 2.5e8, 3) for c, x in v.items()})
    for k, v in j.get("kernels", {}).items():
        if "sample" in k:
            print(f, k[:60], {c: v[c] for c in v if "ns" in c or "count" in c})
PY
