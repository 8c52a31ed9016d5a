# C1 (reference scale, 16k tokens per sweep) work-granule A/B: bench lines at
# tokens_per_range 1/4/8/16(default)/32, then the whole -m gpu suite and smoke
# on the in-tree library.  Everything under gpurun_out/c1tpr/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c1tpr; mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
for tpr in 1 4 8 16 32; do
  timeout -k 10 120 python bench.py --config c1 --no-cpu-baseline --tokens-per-range $tpr > $O/c1_tpr${tpr}_r$rep.log 2>&1 || { echo "c1 tpr $tpr FAILED"; tail -5 $O/c1_tpr${tpr}_r$rep.log; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c1_tpr${tpr}_r$rep.log').read().strip().splitlines()[-1]);print('tpr $tpr', round(d['value']/1e6,1),'Mtok/s', round(d['ms_per_step']*1e3,1),'us/sweep', round(d['roofline']['kernel_ms_timed_region']*1e3,1),'us kernel')"
done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; tail -60 $O/pytest_gpu.log; exit 1; }
echo "pytest: $(grep -E 'passed|failed' $O/pytest_gpu.log | tail -1)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
