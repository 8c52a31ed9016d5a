# Half-wave dense sampler (K <= 128): the whole -m gpu suite, then C2 / C1
# bench lines for the in-tree library and the full-wave variant.
set -o pipefail
shopt -s nullglob
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/half_pytest.log 2>&1 || { echo "PYTEST FAILED"; tail -60 gpurun_out/half_pytest.log; exit 1; }
echo "pytest: $(tail -1 gpurun_out/half_pytest.log)"
for cfg in ${CFGS:-c2 c1}; do
  CFG=$cfg BURNINS="${BURNINS:-0 30}" bash tools/gpu_ab.sh || exit 1
done
