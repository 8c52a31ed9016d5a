# Round 3, step G: large-K sparse sampler A/B (C5 shard): the in-tree library
# against variants (32-bit token offsets; + the batch loop specialised on the
# saturation flag): parity of each (the large-K tests), then C5 at burn-in 0 / 30.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g; mkdir -p $O
export TMPDIR=/tmp
for v in c5v8_nosplit intree; do
  L=$PWD/variants/$v/liblda_mi355x.so; [ $v = intree ] && L=""
  LDA_MI355X_LIB=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_parity_gpu.py -k "sparse or large_k" > $O/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $O/parity_$v.log; exit 1; }
  tail -1 $O/parity_$v.log
done
for b in 0 30; do
  for v in c5base c5v8_nosplit intree; do
    if [ $v = intree ]; then L=""; else L=$PWD/variants/$v/liblda_mi355x.so; fi
    LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --config c5 --burnin $b --no-cpu-baseline > $O/bench_${v}_b$b.log 2>&1 || { echo "BENCH $v $b FAILED"; tail -5 $O/bench_${v}_b$b.log; exit 1; }
    tail -1 $O/bench_${v}_b$b.log > $O/bench_${v}_b$b.jsonl
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_b$b.jsonl').read());r=d['roofline'];print('$v b$b', round(d['value']/1e9,4),'Gtok/s kernel',round(r['kernel_ms_timed_region'],2),'ms')"
  done
done
# the in-tree library: every GPU test, then the reference-scale runs
timeout -k 10 1200 python -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests \
  > $O/pytest_gpu.log 2>&1 || { echo "PYTEST FAILED"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python tools/reference_runs.py > $O/reference_runs.log 2>&1 || { echo "REFRUNS FAILED"; tail -5 $O/reference_runs.log; exit 1; }
cat $O/reference_runs.log
timeout -k 10 300 python tools/estimate_overhead.py > $O/est_overhead.json 2> $O/est_overhead.err || { echo "OVERHEAD FAILED"; tail -5 $O/est_overhead.err; exit 1; }
cat $O/est_overhead.json
for cfg in c1 c1cmu c1ron; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu-baseline > $O/bench_$cfg.log 2>&1 || { echo "BENCH $cfg FAILED"; tail -5 $O/bench_$cfg.log; exit 1; }
  tail -1 $O/bench_$cfg.log > $O/bench_$cfg.jsonl
  python3 -c "import json;d=json.loads(open('$O/bench_$cfg.jsonl').read());r=d['roofline'];print('$cfg', round(d['value']/1e6,1),'Mtok/s', round(d['ms_per_step']*1e3,1),'us/step kernel',round(r['kernel_ms_timed_region']*1e3,1),'us')"
done
PASSES="kt" LABEL=c1ron BENCH_ARGS="--config c1ron" STEPS=100 bash tools/profile.sh > $O/profile_c1ron.log 2>&1 || { echo "PROFILE c1ron FAILED"; tail -10 $O/profile_c1ron.log; exit 1; }
mkdir -p $O/prof_c1ron && cp gpurun_out/prof_c1ron/summary_kt.json gpurun_out/prof_c1ron/*kernel_stats.csv $O/prof_c1ron/ 2>/dev/null
python3 -c "
import json; d=json.load(open('$O/prof_c1ron/summary_kt.json'))
for k,v in sorted(d['kernels'].items(), key=lambda kv:-kv[1]['avg_ns']*kv[1]['calls'])[:8]: print(k, v['calls'], round(v['avg_ns']/1e3,1), 'us avg')
"
