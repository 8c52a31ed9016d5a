# One-document inference latency: in-tree library vs variants/headcapi (tools/infer_latency.py);
# then the inference parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_topic_model_gpu.py -x -q -k "infer" --timeout 200 --timeout-method thread > gpurun_out/infer_parity.log 2>&1 || { echo "PARITY FAILED"; tail -30 gpurun_out/infer_parity.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/infer_parity.log)"
PYTHONPATH=$PWD timeout -k 10 300 python tools/infer_latency.py > gpurun_out/infer_lat_new.json 2> gpurun_out/infer_lat_new.log || { echo NEW FAILED; tail gpurun_out/infer_lat_new.log; exit 1; }
echo "new: $(cat gpurun_out/infer_lat_new.json)"
LDA_MI355X_LIB=$PWD/variants/headcapi/liblda_mi355x.so PYTHONPATH=$PWD timeout -k 10 300 python tools/infer_latency.py > gpurun_out/infer_lat_head.json 2> gpurun_out/infer_lat_head.log || { echo HEAD FAILED; tail gpurun_out/infer_lat_head.log; exit 1; }
echo "head: $(cat gpurun_out/infer_lat_head.json)"
