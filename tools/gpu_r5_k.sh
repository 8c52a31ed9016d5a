set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5k; mkdir -p $O
bash tools/gpu_r5_c5ab.sh r5k 0 tree || exit 1
bash tools/gpu_r5_var.sh r5kv "LDA_SB_RB=default" tree rl1 rl1ns3 rl1ns3rb8 xnoa || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_jni_harness_gpu.py "tests/test_topic_model_gpu.py::test_staleness_sweeps_bit_exact" > $O/jni_stale.log 2>&1; tail -3 $O/jni_stale.log
for rc in 0 1; do LDA_RECOUNT=$rc timeout -k 10 600 python bench.py --config c2 --no-cpu-baseline > $O/c2_rc$rc.log 2>&1 || { tail -5 $O/c2_rc$rc.log; exit 1; }; python3 -c "import json;d=json.loads(open('$O/c2_rc$rc.log').read().strip().splitlines()[-1]);e=d.get('estimate_side',{});print('c2 rc$rc', round(d['value']/1e9,3), 'side', round(e.get('tokens_per_s',0)/1e9,3), e.get('seconds'))"; done
