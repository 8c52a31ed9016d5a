# Round 3, step AA: the large-K sampler's batch loop without the zero rounds
# that pad a row's last partial batch (SB_REM), with 10 and 8 register rounds:
# parity (large-K / sparse / C5 tests), then C5 at burn-in 0 / 30 against the
# in-tree kernel; c5o32 adds 32-bit row starts (SB_OFF32).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3aa; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms')"; }
for v in c5rem c5rem_rb8 c5o32; do
  LDA_MI355X_LIB=$PWD/variants/$v/liblda_mi355x.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_parity_gpu.py tests/test_fullsize_gpu.py tests/test_exchange_gpu.py -k "sparse or large_k or c5" > $O/parity_$v.log 2>&1 || { echo "PARITY $v FAILED"; tail -20 $O/parity_$v.log; exit 1; }
  echo "$v $(tail -1 $O/parity_$v.log)"
done
for b in 0 30; do
  for v in intree c5rem c5rem_rb8 c5o32; do
    L=""; [ $v != intree ] && L=$PWD/variants/$v/liblda_mi355x.so
    LDA_MI355X_LIB=$L timeout -k 10 400 python bench.py --no-cpu-baseline --config c5 --burnin $b > $O/bench_${v}_b${b}.log 2>&1 || { echo "BENCH $v $b FAILED"; tail -5 $O/bench_${v}_b${b}.log; exit 1; }
    tail -1 $O/bench_${v}_b${b}.log > $O/bench_${v}_b${b}.jsonl
    line $O/bench_${v}_b${b}.jsonl "c5 $v b$b"
  done
done
