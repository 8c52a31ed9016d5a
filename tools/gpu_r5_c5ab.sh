# Round-5 C5 A/B: large-K parity tests on the tree's library, then the C5
# bench near init and after 30 burn-in sweeps for each library given
# (path or "tree").  bash tools/gpu_r5_c5ab.sh OUT [TESTS=1] lib...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1; shift
T=$1; shift
mkdir -p $O
if [ "$T" = "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_parity_gpu.py -k "large_k or sparse" > $O/pytest_bigk.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $O/pytest_bigk.log; exit 1; }
  tail -3 $O/pytest_bigk.log
fi
for lib in "$@"; do
  n=$(basename $(dirname $lib))
  [ "$lib" = "tree" ] && n=tree
  for bi in 0 30; do
    if [ "$lib" = "tree" ]; then
      timeout -k 10 600 python bench.py --config c5 --burnin $bi --no-cpu-baseline --no-estimate --dropin-steps 0 > $O/c5_${n}_b$bi.log 2>&1 || { echo "BENCH $n $bi FAILED"; tail -5 $O/c5_${n}_b$bi.log; exit 1; }
    else
      LDA_MI355X_LIB=$lib timeout -k 10 600 python bench.py --config c5 --burnin $bi --no-cpu-baseline --no-estimate --dropin-steps 0 > $O/c5_${n}_b$bi.log 2>&1 || { echo "BENCH $n $bi FAILED"; tail -5 $O/c5_${n}_b$bi.log; exit 1; }
    fi
    python3 -c "import json;d=json.loads(open('$O/c5_${n}_b$bi.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$n b$bi', round(d['value']/1e9,4),'Gtok/s kernel ms',round(r['kernel_ms_timed_region'],3),'frac',round(r['frac'],3))"
  done
done
