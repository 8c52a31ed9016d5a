# Round 3, step A: the recount count update -- parity (recount + delta
# modes, the existing dense parity and config tests) and an A/B of the two
# modes on C2 / C3 / C4-shard at burn-in 0 and 30.  Output: gpurun_out/r3a/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3a; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_recount_gpu.py tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_exchange_gpu.py \
  tests/test_distributed_gpu.py tests/test_abi_guard.py tests/test_topic_model_gpu.py tests/test_jni_harness_gpu.py > $O/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for K in 20 100; do
  timeout -k 10 400 python tools/ppl_gpu_seeds.py $K 1 96 2,0 > $O/ppl_gpu_k$K.json 2> $O/ppl_gpu_k$K.err || { echo "PPL $K FAILED"; tail -5 $O/ppl_gpu_k$K.err; exit 1; }
  cat $O/ppl_gpu_k$K.err
done
for cfg in c2 c3 c4; do
  for b in 0 30; do
    for m in 1 0; do
      LDA_RECOUNT=$m timeout -k 10 300 python bench.py --config $cfg --burnin $b --no-cpu-baseline > $O/bench_${cfg}_b${b}_r${m}.log 2>&1 || { echo "BENCH $cfg $b $m FAILED"; tail -5 $O/bench_${cfg}_b${b}_r${m}.log; exit 1; }
      tail -1 $O/bench_${cfg}_b${b}_r${m}.log > $O/bench_${cfg}_b${b}_r${m}.jsonl
      python3 -c "import json;d=json.loads(open('$O/bench_${cfg}_b${b}_r${m}.jsonl').read());r=d['roofline'];print('$cfg b$b recount=$m', round(d['value']/1e9,3),'Gtok/s', round(d['ms_per_step'],3),'ms/step kernel',round(r['kernel_ms_timed_region'],3),'recount',r.get('recount_ms_timed_region'),'frac',round(r['frac'],3))"
    done
  done
done
