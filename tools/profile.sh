# rocprofv3 passes over one bench command; summaries under gpurun_out/prof_<label>/
# usage: LABEL=x BENCH_ARGS="--config c5" bash tools/profile.sh
# The command is the bench's own (its --steps / --warmup / --burnin, default
# 10 / 3 / 0), and the summaries skip each kernel's first burnin + warmup
# dispatches and keep the next --steps, so the counters and durations
# describe the bench's timed sweeps (--no-estimate: the side figure's
# estimate() runs after the timed region and would dilute the averages).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
P=gpurun_out/prof_${LABEL:-run}
mkdir -p $P
STEPS=${STEPS:-10}; WARMUP=${WARMUP:-3}; BURNIN=${BURNIN:-0}
B="python3 bench.py --steps $STEPS --warmup $WARMUP --burnin $BURNIN --no-cpu-baseline --no-estimate --dropin-steps 0 ${BENCH_ARGS:-}"
SKIP=$((WARMUP + BURNIN))
PER_SWEEP=${PER_SWEEP:-1}   # sampler launches per sweep (--exchange-parts P: P)
SEL='--kernel-include-regex k_sample|k_apply|k_prepare|k_count|k_build|k_recount'
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" -d $P/$name -o $name --output-format csv -- $B > $P/$name.log 2>&1 || { echo "$name FAILED"; tail -20 $P/$name.log; return 1; }
  python3 tools/summarize_prof.py $P/$name $P/summary_$name.json $SKIP $PER_SWEEP $STEPS && cp $P/$name/*kernel_stats.csv $P/ 2>/dev/null; rm -rf $P/$name
  echo "$name ok"
}
PASSES=${PASSES:-"kt fetch write sq lat tcc ea lds"}
ok=0
for p in $PASSES; do
  case $p in
    kt) run kt --kernel-trace --stats ;;
    fetch) run fetch $SEL --pmc FETCH_SIZE ;;
    write) run write $SEL --pmc WRITE_SIZE ;;
    sq) run sq $SEL --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU ;;
    lat) run lat $SEL --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES ;;
    tcc) run tcc $SEL --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum ;;
    ea) run ea $SEL --pmc TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_avr ;;
    lds) run lds $SEL --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS ;;
    grbm) run grbm $SEL --pmc GRBM_GUI_ACTIVE GRBM_COUNT ;;
    sq2) run sq2 $SEL --pmc SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES ;;
  esac || { ok=1; break; }
done
ls $P
exit $ok
