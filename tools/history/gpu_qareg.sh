# A/B of the quarter-wave kernel's register-resident a values (QUARTER_AREG=1,
# variants/qareg) against the in-tree library: the variant's parity on every
# quarter-wave test (variant tests, goldens, C2 workload), then C2 bench lines
# at burn-in 0 and 30 for both libraries.  Everything under gpurun_out/qareg/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/qareg; mkdir -p $O
export TMPDIR=/tmp
LDA_MI355X_LIB=$PWD/variants/qareg/liblda_mi355x.so timeout -k 10 400 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py tests/test_configs_gpu.py -x -q -k "half_wave_variant or golden or c2_c3" --timeout 300 --timeout-method thread > $O/parity_qareg.log 2>&1 || { echo "PARITY FAILED"; tail -40 $O/parity_qareg.log; exit 1; }
echo "qareg parity: $(tail -1 $O/parity_qareg.log)"
CFG=c2 BURNINS="0 30" bash tools/gpu_ab.sh || exit 1
mv gpurun_out/ab_*_b*.log $O/
CFG=c2 BURNINS="0 30" bash tools/gpu_ab.sh || exit 1
