package cmu_gpu;

import java.io.IOException;
import java.util.logging.Logger;

import cc.mallet.topics.ParallelTopicModel;
import cc.mallet.topics.TopicAssignment;
import cc.mallet.types.Dirichlet;
import cc.mallet.types.FeatureSequence;
import cc.mallet.types.LabelSequence;

/**
 * Drop-in for cc.mallet.topics.ParallelTopicModel whose estimate() runs the
 * collapsed-Gibbs sweeps on an MI355X through liblda_mi355x.so (C ABI:
 * include/lda_mi355x.h).  Replace
 *   new ParallelTopicModel(500, 100, 1)   (src/cmu_ron/TrainAndPredict.java:160)
 *   new ParallelTopicModel(100, 10, 0.001) (src/cmu/TrainAndPredict.java:259)
 * with new GpuParallelTopicModel(...); everything downstream
 * (getTopicProbabilities, modelLogLikelihood, getInferencer, printTopWords,
 * printDocumentTopics, Java serialization) reads the Mallet fields this class
 * writes back after the sweeps.
 *
 * Written against Mallet 2.0.7 (pom.xml:107-111).  NOT compiled in the build
 * image (no JDK); see INTEGRATION.md.
 */
public class GpuParallelTopicModel extends ParallelTopicModel {
  private static final Logger logger = Logger.getLogger(GpuParallelTopicModel.class.getName());
  static { System.loadLibrary("lda_mi355x_jni"); }

  private int device = 0;

  public GpuParallelTopicModel(int numberOfTopics, double alphaSum, double beta) {
    super(numberOfTopics, alphaSum, beta);
  }

  public void setDevice(int device) { this.device = device; }

  // --- JNI (integration/jni/lda_jni.c) -------------------------------------
  private static native long nativeCreate(int K, int V, long[] docOff, int[] words, int[] z,
                                          double[] alpha, double beta, long seed, int device);
  private static native void nativeSweep(long ctx, int n);
  private static native void nativeGetZ(long ctx, int[] z);
  private static native void nativeSetAlphaBeta(long ctx, double[] alpha, double beta);
  private static native double nativeLogLikelihood(long ctx);
  /** packed rows (count << topicBits | topic), row offsets [V+1] */
  private static native void nativeMalletPacked(long ctx, int[] rows, long[] rowOff);
  private static native void nativeGetTokensPerTopic(long ctx, int[] tokensPerTopic);
  /** adds docLengthCounts[maxLen+1] and topicDocCounts[K*(maxLen+1)] (flattened) */
  private static native void nativeDocTopicHistograms(long ctx, int maxLen, int[] docLen,
                                                      int[] topicDocFlat);
  /** adds countHistogram[maxCount+1] of the nw cells */
  private static native void nativeCountHistogram(long ctx, long maxCount, int[] hist);
  private static native void nativeDestroy(long ctx);

  @Override
  public void estimate() throws IOException {
    final int D = data.size();
    long[] docOff = new long[D + 1];
    for (int d = 0; d < D; d++) {
      FeatureSequence fs = (FeatureSequence) data.get(d).instance.getData();
      docOff[d + 1] = docOff[d] + fs.getLength();
    }
    final int N = (int) docOff[D];
    int[] words = new int[N];
    int[] z = new int[N];
    for (int d = 0; d < D; d++) {
      TopicAssignment t = data.get(d);
      FeatureSequence fs = (FeatureSequence) t.instance.getData();
      int[] topics = t.topicSequence.getFeatures();
      for (int i = 0; i < fs.getLength(); i++) {
        words[(int) docOff[d] + i] = fs.getIndexAtPosition(i);
        z[(int) docOff[d] + i] = topics[i];          // addInstances' random init is kept
      }
    }
    long seed = randomSeed == -1 ? System.nanoTime() : randomSeed;
    long ctx = nativeCreate(numTopics, numTypes, docOff, words, z, alpha, beta, seed, device);
    int maxLen = 0;
    for (int d = 0; d < D; d++) maxLen = Math.max(maxLen, (int) (docOff[d + 1] - docOff[d]));
    int[] docLen = new int[maxLen + 1];
    int[] topicDocFlat = new int[numTopics * (maxLen + 1)];
    int maxTypeCount = 0;
    for (int w = 0; w < numTypes; w++) maxTypeCount = Math.max(maxTypeCount, typeTotals[w]);
    try {
      for (int iteration = 1; iteration <= numIterations; iteration++) {
        nativeSweep(ctx, 1);
        boolean opt = iteration > burninPeriod && optimizeInterval != 0;
        if (opt && iteration % saveSampleInterval == 0) {
          nativeDocTopicHistograms(ctx, maxLen, docLen, topicDocFlat);   // collectAlphaStatistics
        }
        if (opt && iteration % optimizeInterval == 0) {
          // optimizeAlpha: Mallet's own estimator on the GPU's histograms
          int[][] topicDoc = new int[numTopics][];
          for (int k = 0; k < numTopics; k++) {
            topicDoc[k] = java.util.Arrays.copyOfRange(topicDocFlat, k * (maxLen + 1), (k + 1) * (maxLen + 1));
          }
          if (usingSymmetricAlpha) {
            int[] pooled = new int[maxLen + 1];
            for (int k = 0; k < numTopics; k++)
              for (int i = 0; i <= maxLen; i++) pooled[i] += topicDoc[k][i];
            alphaSum = Dirichlet.learnSymmetricConcentration(pooled, docLen, numTopics, alphaSum);
            java.util.Arrays.fill(alpha, alphaSum / numTopics);
          } else {
            alphaSum = Dirichlet.learnParameters(alpha, topicDoc, docLen, 1.001, 1.0, 1);
          }
          java.util.Arrays.fill(docLen, 0);
          java.util.Arrays.fill(topicDocFlat, 0);
          // optimizeBeta: countHistogram from the GPU, topic sizes from tokensPerTopic
          int[] countHistogram = new int[maxTypeCount + 1];
          nativeCountHistogram(ctx, maxTypeCount, countHistogram);
          nativeGetTokensPerTopic(ctx, tokensPerTopic);
          int maxTopicSize = 0;
          for (int k = 0; k < numTopics; k++) maxTopicSize = Math.max(maxTopicSize, tokensPerTopic[k]);
          int[] topicSizeHistogram = new int[maxTopicSize + 1];
          for (int k = 0; k < numTopics; k++) topicSizeHistogram[tokensPerTopic[k]]++;
          betaSum = Dirichlet.learnSymmetricConcentration(countHistogram, topicSizeHistogram, numTypes, betaSum);
          beta = betaSum / numTypes;
          nativeSetAlphaBeta(ctx, alpha, beta);
        }
        if (iteration % 10 == 0) {
          logger.info("<" + iteration + "> LL/token: " + nativeLogLikelihood(ctx) / N);
        }
      }
      // write the sampler state back into Mallet's fields
      nativeGetZ(ctx, z);
      for (int d = 0; d < D; d++) {
        int[] topics = data.get(d).topicSequence.getFeatures();
        System.arraycopy(z, (int) docOff[d], topics, 0, topics.length);
      }
      long[] rowOff = new long[numTypes + 1];
      int[] rows = new int[0];
      nativeMalletPacked(ctx, null, rowOff);
      rows = new int[(int) rowOff[numTypes]];
      nativeMalletPacked(ctx, rows, rowOff);
      for (int w = 0; w < numTypes; w++) {
        int[] dst = typeTopicCounts[w];               // length min(K, typeTotal), as allocated
        java.util.Arrays.fill(dst, 0);
        System.arraycopy(rows, (int) rowOff[w], dst, 0, (int) (rowOff[w + 1] - rowOff[w]));
      }
      nativeGetTokensPerTopic(ctx, tokensPerTopic);
    } finally {
      nativeDestroy(ctx);
    }
  }
}
