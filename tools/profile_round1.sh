# rocprofv3 passes over the default bench workload (C4 shard, K=512).
# Kernel trace + stats first, then one --pmc pass per counter group
# (FETCH_SIZE and WRITE_SIZE in separate passes: TCC slot limits).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/prof
mkdir -p $P
rocprofv3 -L > $P/counters_list.txt 2>&1 || true
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline"
SEL='--kernel-include-regex k_sample|k_apply|k_prepare|k_count'
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" -d $P/$name -o $name --output-format csv -- $B > $P/$name.log 2>&1 || { echo "$name FAILED"; tail -20 $P/$name.log; return 1; }
  python3 tools/summarize_prof.py $P/$name $P/summary_$name.json && cp $P/$name/*kernel_stats.csv $P/ 2>/dev/null; rm -rf $P/$name
  echo "$name ok"
}
run kt --kernel-trace --stats &&
run fetch $SEL --pmc FETCH_SIZE &&
run write $SEL --pmc WRITE_SIZE &&
run sq $SEL --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU &&
run tcc $SEL --pmc TCC_HIT_sum TCC_MISS_sum &&
run lds $SEL --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
ls -la $P
