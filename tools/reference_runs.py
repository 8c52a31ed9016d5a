"""The reference's own training runs at their own scale, end to end:
ParallelTopicModel.estimate() with the settings of src/cmu/TrainAndPredict.java:259-263
(K=100, alphaSum 10, beta 0.001, 1000 sweeps, optimizeInterval 20) and
src/cmu_ron/TrainAndPredict.java:160-165 (K=500, alphaSum 100, beta 1, 10000
sweeps, optimizeInterval 20), 4 threads, on the C1 changelist-shaped corpus:
the native GPU ParallelTopicModel vs cpu_mallet (oracle/, the Mallet 2.0.7
restatement; a reported baseline).  Usage: python tools/reference_runs.py [sweep_scale]"""
import sys, time
import numpy as np
sys.path.insert(0, '.')
from ldagibbssampling_amd.corpus import synthetic_changelists
from ldagibbssampling_amd import topic_model as tm
from oracle import oracle as O

scale = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
c = synthetic_changelists()
# untimed: the HIP runtime and the kernels' code objects load on the process's
# first GPU call (~2 s on a fresh box), which is not the estimate()
w = tm.ParallelTopicModel(100, 10.0, 0.01)
w.addInstances(tm.InstanceList.fromCorpus(c))
w.setTopicDisplay(0, 0)
w.setNumIterations(2)
w.estimate()
del w
for name, K, asum, beta, sweeps in [("src/cmu", 100, 10.0, 0.001, 1000), ("src/cmu_ron", 500, 100.0, 1.0, 10000)]:
    sweeps = int(sweeps * scale)
    m = tm.ParallelTopicModel(K, asum, beta)
    m.addInstances(tm.InstanceList.fromCorpus(c))
    m.setRandomSeed(1)
    m.setTopicDisplay(0, 0)
    m.setOptimizeInterval(20)
    m.setNumThreads(4)
    m.setNumIterations(sweeps)
    t = time.perf_counter()
    m.estimate()
    tg = time.perf_counter() - t
    llg = m.modelLogLikelihood() / c.num_tokens
    mm = O.MalletModel(K, asum, beta, c.num_types, c.doc_off, c.words, seed=1, num_threads=4)
    mm.set_optimize(20, burnin=200)
    t = time.perf_counter()
    mm.estimate(sweeps)
    tc = time.perf_counter() - t
    print(f"{name}: K={K} {sweeps} sweeps over {c.num_tokens} tokens ({c.num_docs} docs): GPU ParallelTopicModel "
          f"{tg:.2f} s (LL/token {llg:.4f}, incl. LL every 10 sweeps and alpha/beta optimisation) | cpu_mallet 4 threads "
          f"{tc:.2f} s (LL/token {mm.log_likelihood()/c.num_tokens:.4f}) | {tc/tg:.1f}x", flush=True)
