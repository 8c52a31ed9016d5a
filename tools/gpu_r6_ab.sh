# Round 6, GPU call AB: C5 work-range size (bench --tokens-per-range: the
# library's default is ~32 ranges per wave, 1907 tokens here) near init and
# after 30 sweeps, both orders.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ab; mkdir -p $O
for pass in a b; do
  L="0 950 3800 600"; [ $pass = b ] && L="600 3800 950 0"
  for tpr in $L; do
    for bi in 0 30; do
      timeout -k 10 600 python bench.py --config c5 --burnin $bi --no-cpu-baseline --no-estimate --dropin-steps 0 \
        --tokens-per-range $tpr > $O/c5_${pass}_tpr${tpr}_b$bi.log 2>&1 || { tail -5 $O/c5_${pass}_tpr${tpr}_b$bi.log; exit 1; }
      python3 -c "import json;d=json.loads(open('$O/c5_${pass}_tpr${tpr}_b$bi.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$pass tpr $tpr b$bi', round(d['value']/1e9,4), round(r['kernel_ms_timed_region'],3))"
    done
  done
done
