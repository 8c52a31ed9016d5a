# Round 3, step B: the recount kernel without a work queue -- parity of both
# count-update modes, the change rate per sweep, and the A/B on C2 / C4-shard.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r3b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_recount_gpu.py > $O/pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python tools/change_rate.py c2 40 > $O/change_c2.json 2> $O/change_c2.err || { echo "CHANGE c2 FAILED"; tail -5 $O/change_c2.err; exit 1; }
timeout -k 10 300 python tools/change_rate.py c4 40 312500 > $O/change_c4q.json 2> $O/change_c4q.err || { echo "CHANGE c4 FAILED"; tail -5 $O/change_c4q.err; exit 1; }
for cfg in c2 c4; do
  for b in 0 30; do
    for m in 1 0; do
      LDA_RECOUNT=$m timeout -k 10 300 python bench.py --config $cfg --burnin $b --no-cpu-baseline > $O/bench_${cfg}_b${b}_r${m}.log 2>&1 || { echo "BENCH $cfg $b $m FAILED"; tail -5 $O/bench_${cfg}_b${b}_r${m}.log; exit 1; }
      tail -1 $O/bench_${cfg}_b${b}_r${m}.log > $O/bench_${cfg}_b${b}_r${m}.jsonl
      python3 -c "import json;d=json.loads(open('$O/bench_${cfg}_b${b}_r${m}.jsonl').read());r=d['roofline'];print('$cfg b$b recount=$m', round(d['value']/1e9,3),'Gtok/s', round(d['ms_per_step'],3),'ms/step kernel',round(r['kernel_ms_timed_region'],3),'recount',r.get('recount_ms_timed_region'),'frac',round(r['frac'],3))"
    done
  done
done
python3 -c "
import json
for f in ('$O/change_c2.json','$O/change_c4q.json'):
    d=json.load(open(f)); print(f, [round(x,3) for x in d['changed_fraction_per_sweep']])
"
