# FETCH_SIZE / WRITE_SIZE calibration on known byte counts (tools/fetch_calib.hip),
# one rocprofv3 pass per counter; result in gpurun_out/calib/fetch_calib.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/calib; mkdir -p $O
timeout -k 10 120 ./tools/bin/fetch_calib > $O/known.json 2> $O/known.log || { echo "CALIB RUN FAILED"; cat $O/known.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | tr A-Z a-z | cut -d_ -f1)
  timeout -s KILL 120 rocprofv3 --pmc $c -d $O/$n -o $n --output-format csv -- ./tools/bin/fetch_calib > $O/$n.log 2>&1 || { echo "PMC $c FAILED"; tail -20 $O/$n.log; exit 1; }
  python3 tools/summarize_prof.py $O/$n $O/summary_$n.json && rm -rf $O/$n
done
python3 tools/fetch_calib.py $O/known.json $O/summary_fetch.json $O/summary_write.json $O/fetch_calib.json
