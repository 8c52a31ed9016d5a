# Round 3, step AD: the dense sampler's per-token document-count update with
# both counts read before either is written (one LDS round trip instead of two
# dependent ones, LDA_ND_ONETRIP; the variant also carries the large-K
# sampler's no-return count atomics): parity (dense tests), then the C4 shard,
# C3 and the whole-C4 default line against the in-tree library.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3ad; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms')"; }
v=c4one
LDA_MI355X_LIB=$PWD/variants/$v/liblda_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_exchange_gpu.py tests/test_graph_gpu.py > $O/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $O/parity_$v.log; exit 1; }
echo "$v $(tail -1 $O/parity_$v.log)"
for rep in 1 2; do
  for cfg in c4shard c3; do
    for v in intree c4one; do
      L=""; [ $v != intree ] && L=$PWD/variants/$v/liblda_mi355x.so
      LDA_MI355X_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --config $cfg > $O/bench_${v}_${cfg}_$rep.log 2>&1 || { echo "BENCH $v $cfg FAILED"; tail -5 $O/bench_${v}_${cfg}_$rep.log; exit 1; }
      tail -1 $O/bench_${v}_${cfg}_$rep.log > $O/bench_${v}_${cfg}_$rep.jsonl
      line $O/bench_${v}_${cfg}_$rep.jsonl "$cfg $v rep$rep"
    done
  done
done
for v in intree c4one; do
  L=""; [ $v != intree ] && L=$PWD/variants/$v/liblda_mi355x.so
  LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench_${v}_default.log 2>&1 || { echo "BENCH $v default FAILED"; tail -5 $O/bench_${v}_default.log; exit 1; }
  tail -1 $O/bench_${v}_default.log > $O/bench_${v}_default.jsonl
  line $O/bench_${v}_default.jsonl "default $v"
done
