# Round 3, step H: graph-launched sweeps (lda_sweep / estimate()) — every GPU
# test, the reference-scale runs with and without graphs; then the static
# first work range A/B (variants/nostatic) on C2 and C4 at burn-in 0 / 30.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3h; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs.log 2>&1 || { echo "REFRUNS FAILED"; tail -5 $O/reference_runs.log; exit 1; }
cat $O/reference_runs.log
LDA_GRAPHS=0 timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs_nograph.log 2>&1 || { echo "REFRUNS nograph FAILED"; tail -5 $O/reference_runs_nograph.log; exit 1; }
cat $O/reference_runs_nograph.log
timeout -k 10 300 python tools/estimate_overhead.py > $O/est_overhead.json 2> $O/est_overhead.err || { echo "OVERHEAD FAILED"; tail -5 $O/est_overhead.err; exit 1; }
cat $O/est_overhead.json
for cfg in c2 c4; do
  for b in 0 30; do
    for v in nostatic intree; do
      if [ $v = intree ]; then L=""; else L=$PWD/variants/$v/liblda_mi355x.so; fi
      LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --config $cfg --burnin $b --no-cpu-baseline > $O/bench_${cfg}_${v}_b$b.log 2>&1 || { echo "BENCH $cfg $v $b FAILED"; tail -5 $O/bench_${cfg}_${v}_b$b.log; exit 1; }
      tail -1 $O/bench_${cfg}_${v}_b$b.log > $O/bench_${cfg}_${v}_b$b.jsonl
      python3 -c "import json;d=json.loads(open('$O/bench_${cfg}_${v}_b$b.jsonl').read());r=d['roofline'];print('$cfg $v b$b', round(d['value']/1e9,4),'Gtok/s kernel',round(r['kernel_ms_timed_region'],2),'ms')"
    done
  done
done
