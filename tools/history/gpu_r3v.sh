# Round 3, step V: the large-K register rounds and round count bounded by a tier of the row length (SB_TIER) against the in-tree kernel on C5.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3v; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms')"; }
LDA_MI355X_LIB=$PWD/variants/c5tier/liblda_mi355x.so timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_parity_gpu.py -k "sparse or large_k" > $O/parity.log 2>&1 || { echo "PARITY FAILED"; tail -20 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for b in 0 30; do for v in intree c5tier intree c5tier; do
  L=""; [ $v != intree ] && L=$PWD/variants/$v/liblda_mi355x.so
  LDA_MI355X_LIB=$L timeout -k 10 600 python bench.py --no-cpu-baseline --config c5 --burnin $b > $O/b.log 2>&1 || { echo "BENCH FAILED"; tail -5 $O/b.log; exit 1; }
  tail -1 $O/b.log > $O/b.jsonl; line $O/b.jsonl "c5 $v b$b"
done; done
