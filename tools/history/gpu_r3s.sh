# Round 3, step S: with the word-ordered z copy, does the recount still lose
# to the delta after burn-in?  C2 at burn-in 30 and 100: default AUTO (delta
# after 20 sweeps) against LDA_RECOUNT=1 (every sweep recounts), two repeats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3s; mkdir -p $O
export TMPDIR=/tmp
line() { python3 -c "import json;d=json.loads(open('$1').read());r=d['roofline'];print('$2', round(d['value']/1e9,4),'Gtok/s', round(d['ms_per_step'],4), 'ms/step kernel',round(r['kernel_ms_timed_region'],4),'ms recount', r.get('recount_ms_timed_region'))"; }
for b in 30 100; do
  for rep in 1 2; do
    for m in auto recount; do
      if [ $m = recount ]; then E="LDA_RECOUNT=1"; else E="LDA_RECOUNT=x"; fi
      env $E timeout -k 10 600 python bench.py --no-cpu-baseline --config c2 --burnin $b > $O/bench_${m}_b${b}_$rep.log 2>&1 || { echo "BENCH $m $b FAILED"; tail -5 $O/bench_${m}_b${b}_$rep.log; exit 1; }
      tail -1 $O/bench_${m}_b${b}_$rep.log > $O/bench_${m}_b${b}_$rep.jsonl
      line $O/bench_${m}_b${b}_$rep.jsonl "c2 $m b$b rep$rep"
    done
  done
done
