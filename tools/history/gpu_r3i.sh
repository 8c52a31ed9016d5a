# Round 3, step I: the wave-uniform work-range index (in-tree) against the
# static-first build without it (variants/nostatic = no static first range,
# variants/c5head = the previous commit) on C4/C3/C2; the large-K sampler's
# scalar-work variants on C5 at burn-in 0 / 30; the C1 range floor.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3i; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_graph_gpu.py \
  > $O/graph_tests.log 2>&1 || { echo "GRAPH TESTS FAILED"; tail -30 $O/graph_tests.log; exit 1; }
tail -1 $O/graph_tests.log
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms')"; }
run() {  # run NAME VARIANT ARGS...
  local n=$1 v=$2; shift 2
  local L=""; [ $v != intree ] && L=$PWD/variants/$v/liblda_mi355x.so
  LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --no-cpu-baseline "$@" > $O/bench_$n.log 2>&1 || { echo "BENCH $n FAILED"; tail -5 $O/bench_$n.log; exit 1; }
  tail -1 $O/bench_$n.log > $O/bench_$n.jsonl
  line $O/bench_$n.jsonl $n
}
for b in 0 30; do run c4_intree_b$b intree --config c4 --burnin $b; done
run c3_intree_b0 intree --config c3
run c3_nostatic_b0 nostatic --config c3
run c2_intree_b0 intree --config c2
for tpr in 8 12 16; do run c1ron_tpr$tpr intree --config c1ron --tokens-per-range $tpr; done
for b in 0 30; do
  for v in c5head intree c5u c5uv c5ut c5uvt c5w12 c5w12vt c5ns2 c5rb8; do
    run c5_${v}_b$b $v --config c5 --burnin $b
  done
done
