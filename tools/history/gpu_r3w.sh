# Round 3, step W: the final library once more as the driver runs it (every
# GPU test, smoke()), then a kernel trace of the reference's two training
# runs end to end (tools/reference_runs.py: graph-launched sweeps, LL logs,
# optimisation), whose per-kernel statistics go to profiles/r03/graph/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3w; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_ref -o kt --output-format csv -- python3 tools/reference_runs.py > $O/reference_runs_prof.log 2>&1 || { echo "PROFILED REFRUNS FAILED"; tail -20 $O/reference_runs_prof.log; exit 1; }
grep -E "^src/" $O/reference_runs_prof.log
find $O/prof_ref -name "*kernel_stats.csv" -exec cp {} $O/ref_kernel_stats.csv \;
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r3w/ref_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us avg", round(float(r["TotalDurationNs"]) / 1e6, 1), "ms total")
PY
