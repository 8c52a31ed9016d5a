set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r5x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_exchange_gpu.py tests/test_distributed_gpu.py "tests/test_parity_gpu.py::test_large_k_ring_probe_with_empty_first_part" "tests/test_topic_model_gpu.py::test_shard_group_compact_exchange_on_one_device" "tests/test_topic_model_gpu.py::test_shard_group_on_one_device" > $O/xch.log 2>&1; rc=$?; tail -4 $O/xch.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_r5_k.sh
