# Round 6, GPU call C: the C2 packed-fp32 A/B (variants/qpk, -DQUARTER_PK=1:
# quarter parity on it, then C2 near init / after 30 sweeps against the
# tree), the C2 profile, the large-K perplexity statistics (-s), a 2-rank
# rehearsal of the default bench over gloo on one GPU (count staging, the
# drop-in schedule line), and last the per-path counts of the large-K draw
# (variants/xcount, -DSB_X_COUNT=1: the round-5 null-trace fault's fix).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c; mkdir -p $O
LDA_MI355X_LIB=variants/qpk/liblda_mi355x.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 \
  --timeout-method thread -m gpu tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_recount_gpu.py \
  -k "quarter or sweeps_bit_exact or c2 or recount" > $O/qpk_parity.log 2>&1 || { tail -20 $O/qpk_parity.log; exit 1; }
tail -1 $O/qpk_parity.log
for bi in 0 30; do
  for lib in tree qpk; do
    if [ $lib = tree ]; then L=""; else L=variants/qpk/liblda_mi355x.so; fi
    LDA_MI355X_LIB=$L timeout -k 10 300 python bench.py --config c2 --burnin $bi --no-cpu-baseline --no-estimate --dropin-steps 0 > $O/c2_${lib}_b$bi.log 2>&1 || { tail -5 $O/c2_${lib}_b$bi.log; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c2_${lib}_b$bi.log').read().strip().splitlines()[-1]);r=d['roofline'];print('c2 $lib b$bi', round(d['value']/1e9,4),'Gtok/s kernel ms',round(r['kernel_ms_timed_region'],4),'frac',round(r['frac'],3))"
  done
done
LABEL=r6_c2 BENCH_ARGS="--config c2" PASSES="kt fetch write sq lds grbm" bash tools/profile.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -s --timeout 500 --timeout-method thread -m gpu tests/test_perplexity.py \
  -k "2048 or 4096" > $O/ppl_large_k.log 2>&1 || { tail -20 $O/ppl_large_k.log; exit 1; }
grep -E "^K=|GPU_PER_SEED|passed" $O/ppl_large_k.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 \
  bench.py --gpus 2 --steps 4 --warmup 1 --docs 25000 --backend gloo --no-cpu-baseline > $O/bench_2ranks.log 2>&1 \
  || { tail -30 $O/bench_2ranks.log; exit 1; }
grep '^{' $O/bench_2ranks.log | tail -1 > $O/bench_2ranks.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_2ranks.jsonl').read());print('2 ranks', round(d['value']/1e9,3), d['collective']['replicas_agree'], d['dropin_schedule'])"
timeout -k 10 600 python bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
tail -n 1 $O/bench_default.log > $O/bench_default.jsonl
python3 -c "import json;d=json.loads(open('$O/bench_default.jsonl').read());r=d['roofline'];print('default', round(d['value']/1e9,4), 'traffic', r['traffic'], 'issue', (r['issue'] or {}).get('frac'), 'dropin', d['dropin_schedule']['tokens_per_s']/1e9, 'cpu', d['cpu_baseline']['value'])"
LDA_MI355X_LIB=variants/xcount/liblda_mi355x.so timeout -k 10 300 python tools/count_paths.py 300000 0 30 > $O/count_paths.jsonl 2> $O/count_paths.err \
  || { tail -20 $O/count_paths.err; exit 1; }
cat $O/count_paths.jsonl
