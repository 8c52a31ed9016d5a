package cmu_gpu;

import java.io.IOException;
import java.text.DecimalFormat;
import java.util.logging.Logger;

import cc.mallet.topics.ParallelTopicModel;
import cc.mallet.topics.TopicAssignment;
import cc.mallet.types.FeatureSequence;

/**
 * Drop-in for cc.mallet.topics.ParallelTopicModel whose estimate() runs on
 * MI355X GPUs through liblda_mi355x_jni.so (JNI glue: integration/jni/lda_jni.c;
 * native logic: integration/jni/lda_jni_core.c over include/lda_topic_model.h).
 * Replace
 *   new ParallelTopicModel(500, 100, 1)    (src/cmu_ron/TrainAndPredict.java:160)
 *   new ParallelTopicModel(100, 10, 0.001) (src/cmu/TrainAndPredict.java:259)
 * with new GpuParallelTopicModel(...).  estimate() replaces the sweeps, the
 * alpha/beta optimisation and the LL/token log; afterwards the Mallet fields
 * (topicSequence of every document, typeTopicCounts, tokensPerTopic, alpha,
 * alphaSum, beta, betaSum) hold the GPU's state, so getTopicProbabilities,
 * modelLogLikelihood, getInferencer, printTopWords, printDocumentTopics and
 * Java serialization keep working.
 *
 * - setNumThreads(n): Mallet's document blocks become GPU shards
 *   (min(n, visible GPUs)) with an RCCL all-reduce of the count delta per
 *   sweep; the result does not depend on n.
 * - K > 1024 runs the large-K sparse sampler (chosen natively).
 * - The Philox sweep counter is a field of this object (serialized with it):
 *   a second estimate() (updateModel, src/cmu_ron/TrainAndPredict.java:173-177)
 *   continues the random stream instead of replaying the first one's draws.
 *
 * Written against Mallet 2.0.7 (pom.xml:107-111) using only its public fields
 * and setters.  NOT compiled in the build image (no JDK); the native call it
 * makes is compiled and GPU-tested there (tests/jni/estimate_harness.c).
 */
public class GpuParallelTopicModel extends ParallelTopicModel {
  private static final long serialVersionUID = 1L;
  private static final Logger logger = Logger.getLogger(GpuParallelTopicModel.class.getName());

  /**
   * The native library, loaded on the first estimate() only: initialising
   * this class (Java deserialization in the reference's load(),
   * src/cmu_ron/TrainAndPredict.java:191-196, which predict() calls at :246)
   * must work on a host without liblda_mi355x_jni.so, since prediction needs
   * no GPU.  The JVM links the native method when it is first called.
   */
  private static final class NativeLibrary {
    static { System.loadLibrary("lda_mi355x_jni"); }
    static void load() {}
  }

  private int gpuShards = 1;        // setNumThreads
  private long gpuSeed = -1;        // setRandomSeed (-1: time-seeded, as Mallet)
  private long gpuSweep = 0;        // Philox sweep counter carried across estimate() calls
  private int verbosity = 0;

  public GpuParallelTopicModel(int numberOfTopics, double alphaSum, double beta) {
    super(numberOfTopics, alphaSum, beta);
  }

  @Override
  public void setNumThreads(int threads) {
    super.setNumThreads(threads);
    gpuShards = threads;
  }

  @Override
  public void setRandomSeed(int seed) {
    super.setRandomSeed(seed);
    gpuSeed = seed;
  }

  /** 1: the native side prints Mallet's INFO lines on stderr as well. */
  public void setNativeVerbosity(int level) { verbosity = level; }

  /** Largest corpus (tokens) the flat int[] hand-over supports: Integer.MAX_VALUE - 8. */
  public static final long MAX_TOKENS = Integer.MAX_VALUE - 8L;

  // --- JNI (integration/jni/lda_jni.c) -------------------------------------
  private static native int nativeEstimate(int K, int V, long[] docOff, int[] words, int[] z,
                                           double[] alpha, double[] hyper, long[] sweep,
                                           int[] options, long seed, long[] rowOff, int[] rows,
                                           int[] tokensPerTopic, int[] llIter, double[] llValue);

  @Override
  public void estimate() throws IOException {
    NativeLibrary.load();
    final int D = data.size();
    long[] docOff = new long[D + 1];
    for (int d = 0; d < D; d++) {
      FeatureSequence fs = (FeatureSequence) data.get(d).instance.getData();
      docOff[d + 1] = docOff[d] + fs.getLength();
    }
    // Java arrays are int-indexed: the flat token arrays hold at most
    // MAX_TOKENS (the JVM's largest safe array length); a larger corpus
    // needs the native ParallelTopicModel (include/lda_topic_model.h) fed in
    // pieces, not this drop-in (INTEGRATION.md "Limits")
    if (docOff[D] > MAX_TOKENS)
      throw new IllegalArgumentException("corpus has " + docOff[D] + " tokens; GpuParallelTopicModel "
          + "passes them as one Java int[] and supports at most " + MAX_TOKENS);
    final int N = (int) docOff[D];
    int[] words = new int[N];
    int[] z = new int[N];
    for (int d = 0; d < D; d++) {
      TopicAssignment t = data.get(d);
      FeatureSequence fs = (FeatureSequence) t.instance.getData();
      int[] topics = t.topicSequence.getFeatures();
      for (int i = 0; i < fs.getLength(); i++) {
        words[(int) docOff[d] + i] = fs.getIndexAtPosition(i);
        z[(int) docOff[d] + i] = topics[i];          // addInstances' random topics are kept
      }
    }
    // typeTopicCounts rows as addInstances allocated them: min(K, typeTotal)
    long[] rowOff = new long[numTypes + 1];
    for (int w = 0; w < numTypes; w++) rowOff[w + 1] = rowOff[w] + typeTopicCounts[w].length;
    if (rowOff[numTypes] > MAX_TOKENS)
      throw new IllegalArgumentException("typeTopicCounts hold " + rowOff[numTypes] + " cells; at most "
          + MAX_TOKENS + " fit one Java int[]");
    int[] rows = new int[(int) rowOff[numTypes]];
    double[] hyper = {alphaSum, beta, betaSum};
    long[] sweep = {gpuSweep};
    int[] options = {numIterations, burninPeriod, optimizeInterval, saveSampleInterval,
                     usingSymmetricAlpha ? 1 : 0, gpuShards, verbosity};
    long seed = gpuSeed == -1 ? System.nanoTime() : gpuSeed;
    int[] llIter = new int[numIterations / 10 + 1];
    double[] llValue = new double[llIter.length];

    int nll = nativeEstimate(numTopics, numTypes, docOff, words, z, alpha, hyper, sweep, options,
                             seed, rowOff, rows, tokensPerTopic, llIter, llValue);

    DecimalFormat fmt = new DecimalFormat("0.#####");
    for (int i = 0; i < Math.min(nll, llIter.length); i++)
      logger.info("<" + llIter[i] + "> LL/token: " + fmt.format(llValue[i]));
    // write the sampler state back into Mallet's fields
    for (int d = 0; d < D; d++) {
      int[] topics = data.get(d).topicSequence.getFeatures();
      System.arraycopy(z, (int) docOff[d], topics, 0, topics.length);
    }
    for (int w = 0; w < numTypes; w++)
      System.arraycopy(rows, (int) rowOff[w], typeTopicCounts[w], 0, typeTopicCounts[w].length);
    alphaSum = hyper[0];
    beta = hyper[1];
    betaSum = hyper[2];
    gpuSweep = sweep[0];
  }
}
