# Round-5 A/B of kernel variants on C5: for each variants/<name>/liblda_mi355x.so
# (or "tree"), the C5 bench near init and after 30 burn-in sweeps.
#   bash tools/gpu_r5_var.sh OUT "bench env" name...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
ENVS=$1; shift
mkdir -p $O
for n in "$@"; do
  lib=variants/$n/liblda_mi355x.so
  for bi in 0 30; do
    if [ "$n" = "tree" ]; then L=""; else L="LDA_MI355X_LIB=$lib"; fi
    env $ENVS $L timeout -k 10 600 python bench.py --config c5 --burnin $bi --no-cpu-baseline --no-estimate > $O/c5_${n}_b$bi.log 2>&1 || { echo "BENCH $n $bi FAILED"; tail -5 $O/c5_${n}_b$bi.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c5_${n}_b$bi.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$n b$bi', round(d['value']/1e9,4),'Gtok/s kernel ms',round(r['kernel_ms_timed_region'],3))"
  done
done
