# Quarter-wave document counts from the chunk registers: parity of the in-tree
# library on the dense/quarter tests, goldens and the C2 workload, then C1/C2
# bench A/B against variants/base (the previous library).  gpurun_out/qdoc/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/qdoc; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_configs_gpu.py -x -q -k "dense or half_wave_variant or golden or c2_c3 or ragged or edge or empty" --timeout 300 --timeout-method thread > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity.log; exit 1; }
echo "parity: $(tail -1 $O/parity.log)"
for rep in 1 2; do
CFG=c1 BURNINS="0" bash tools/gpu_ab.sh || exit 1
mkdir -p $O/c1_r$rep; mv gpurun_out/ab_*_b*.log $O/c1_r$rep/
done
CFG=c2 BURNINS="0 30" bash tools/gpu_ab.sh || exit 1
mkdir -p $O/c2; mv gpurun_out/ab_*_b*.log $O/c2/
