# Round 3, step D: count-update modes + warm start + async LL + device
# statistics + multi-shard on one GPU -- the affected GPU tests; held-out
# perplexity over 96 seeds with the warm start; the C2/C3 recount crossover.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3d; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_recount_gpu.py tests/test_topic_model_gpu.py tests/test_distributed_gpu.py tests/test_hyper_gpu.py \
  tests/test_parity_gpu.py tests/test_jni_harness_gpu.py tests/test_exchange_gpu.py tests/test_abi_guard.py \
  > $O/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for K in 20 100; do
  timeout -k 10 400 python tools/ppl_gpu_seeds.py $K 1 96 2,0 4,50 > $O/ppl_gpu_warm_k$K.json 2> $O/ppl_gpu_warm_k$K.err || { echo "PPL $K FAILED"; tail -5 $O/ppl_gpu_warm_k$K.err; exit 1; }
  grep seeds $O/ppl_gpu_warm_k$K.err
done
for cfg in c2 c3; do
  for b in 3 7 12 17; do
    for m in 1 0; do
      LDA_RECOUNT=$m timeout -k 10 300 python bench.py --config $cfg --burnin $b --warmup 0 --steps 3 --no-cpu-baseline > $O/bench_${cfg}_b${b}_r${m}.log 2>&1 || { echo "BENCH $cfg $b $m FAILED"; tail -5 $O/bench_${cfg}_b${b}_r${m}.log; exit 1; }
      tail -1 $O/bench_${cfg}_b${b}_r${m}.log > $O/bench_${cfg}_b${b}_r${m}.jsonl
      python3 -c "import json;d=json.loads(open('$O/bench_${cfg}_b${b}_r${m}.jsonl').read());r=d['roofline'];print('$cfg b$b recount=$m', round(d['value']/1e9,3),'Gtok/s', round(d['ms_per_step'],3),'ms/step kernel',round(r['kernel_ms_timed_region'],3),'recount',r.get('recount_ms_timed_region'))"
    done
  done
done
