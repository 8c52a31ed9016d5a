# Perplexity over 12 seeds at K=20 and K=100 (full-wave vs quarter-wave vs cpu_mallet).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/ppl; mkdir -p $O
for K in 20 100; do
  timeout -k 10 500 python -u tools/perplexity_seeds.py $K 1 2 3 4 5 6 7 8 9 10 11 12 > $O/ppl_k$K.json 2> $O/ppl_k$K.log || { echo "PPL K=$K FAILED"; tail -20 $O/ppl_k$K.log; exit 1; }
  tail -3 $O/ppl_k$K.log
done
