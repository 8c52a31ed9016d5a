# Round 3, step P: the dense K = 512 sampler's tuning macros re-checked on
# the C4 shard after the round's changes (vector prefix count, prefetch depth
# 2 / 4, no static first range): parity of each (dense bit-exact tests), then
# the C4 shard at burn-in 0 / 30, two repeats of the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3p; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms')"; }
for v in d_sc0 d_p4 d_p2 d_st0; do
  LDA_MI355X_LIB=$PWD/variants/$v/liblda_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_parity_gpu.py -k "sweeps_bit_exact and dense" > $O/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
for b in 0 30; do
  for v in intree d_sc0 d_p4 d_p2 d_st0 intree; do
    L=""; [ $v != intree ] && L=$PWD/variants/$v/liblda_mi355x.so
    LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --no-cpu-baseline --config c4shard --burnin $b > $O/bench_${v}_b$b.log 2>&1 || { echo "BENCH $v $b FAILED"; tail -5 $O/bench_${v}_b$b.log; exit 1; }
    tail -1 $O/bench_${v}_b$b.log > $O/bench_${v}_b$b.jsonl
    line $O/bench_${v}_b$b.jsonl "c4shard $v b$b"
  done
done
