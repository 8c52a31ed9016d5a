# Round 3, step G: large-K sparse sampler A/B (C5 shard): the in-tree library
# against variants (32-bit token offsets; + the batch loop specialised on the
# saturation flag): parity of each (the large-K tests), then C5 at burn-in 0 / 30.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3g; mkdir -p $O
export TMPDIR=/tmp
for v in c5v8_nosplit c5v8; do
  LDA_MI355X_LIB=$PWD/variants/$v/liblda_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_parity_gpu.py -k "sparse or large_k" > $O/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $O/parity_$v.log; exit 1; }
  tail -1 $O/parity_$v.log
done
for b in 0 30; do
  for v in intree c5v8_nosplit c5v8; do
    if [ $v = intree ]; then L=""; else L=$PWD/variants/$v/liblda_mi355x.so; fi
    LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --config c5 --burnin $b --no-cpu-baseline > $O/bench_${v}_b$b.log 2>&1 || { echo "BENCH $v $b FAILED"; tail -5 $O/bench_${v}_b$b.log; exit 1; }
    tail -1 $O/bench_${v}_b$b.log > $O/bench_${v}_b$b.jsonl
    python3 -c "import json;d=json.loads(open('$O/bench_${v}_b$b.jsonl').read());r=d['roofline'];print('$v b$b', round(d['value']/1e9,4),'Gtok/s kernel',round(r['kernel_ms_timed_region'],2),'ms')"
  done
done
