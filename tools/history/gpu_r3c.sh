# Round 3, step C: where the recount stops paying on C2 / C3 (sweep index of
# the crossover between the two count-update modes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3c; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_recount_gpu.py tests/test_topic_model_gpu.py tests/test_distributed_gpu.py tests/test_hyper_gpu.py tests/test_parity_gpu.py tests/test_jni_harness_gpu.py > $O/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for cfg in c2 c3; do
  for b in 3 7 12 17 22; do
    for m in 1 0; do
      LDA_RECOUNT=$m timeout -k 10 300 python bench.py --config $cfg --burnin $b --warmup 0 --steps 3 --no-cpu-baseline > $O/bench_${cfg}_b${b}_r${m}.log 2>&1 || { echo "BENCH $cfg $b $m FAILED"; tail -5 $O/bench_${cfg}_b${b}_r${m}.log; exit 1; }
      tail -1 $O/bench_${cfg}_b${b}_r${m}.log > $O/bench_${cfg}_b${b}_r${m}.jsonl
      python3 -c "import json;d=json.loads(open('$O/bench_${cfg}_b${b}_r${m}.jsonl').read());r=d['roofline'];print('$cfg b$b recount=$m', round(d['value']/1e9,3),'Gtok/s', round(d['ms_per_step'],3),'ms/step kernel',round(r['kernel_ms_timed_region'],3),'recount',r.get('recount_ms_timed_region'))"
    done
  done
done
