/*
 * lda_jni_core.h — the native half of cmu_gpu.GpuParallelTopicModel.estimate()
 * as plain C over include/lda_topic_model.h (liblda_topic_model.so).
 *
 * The JNI glue (lda_jni.c) only pins the Java arrays and calls ldaj_estimate;
 * everything else the drop-in does natively lives here, so it is compiled
 * and GPU-tested in the build image (tests/jni/estimate_harness.c,
 * tests/test_jni_harness_gpu.py) although jni.h is absent there.
 *
 * Replaces, for the reference's two callers of Mallet 2.0.7's
 * ParallelTopicModel.estimate() (src/cmu_ron/TrainAndPredict.java:166 and
 * :175 (updateModel), src/cmu/TrainAndPredict.java:265 and :273):
 *   - the sweeps (WorkerRunnable.sampleTopicsForOneDoc, numThreads document
 *     blocks -> GPU shards with an RCCL all-reduce of the count delta);
 *   - optimizeAlpha / optimizeBeta on Mallet's schedule;
 *   - the LL/token trace every 10 iterations;
 * and hands back everything Mallet's fields hold afterwards: the topics of
 * every token, the packed typeTopicCounts rows, tokensPerTopic, alpha,
 * alphaSum, beta, betaSum — plus the Philox sweep counter, which the Java
 * object keeps so that the next estimate() continues the random stream.
 */
#ifndef LDA_JNI_CORE_H
#define LDA_JNI_CORE_H

#include <stdint.h>

#include "lda_topic_model.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Mallet's estimate() options, read from the ParallelTopicModel fields. */
typedef struct ldaj_options {
  int32_t num_iterations;       /* numIterations                            */
  int32_t burnin_period;        /* burninPeriod (Mallet default 200)        */
  int32_t optimize_interval;    /* optimizeInterval (0 = off)               */
  int32_t save_sample_interval; /* saveSampleInterval (Mallet default 10)   */
  int32_t symmetric_alpha;      /* usingSymmetricAlpha                      */
  int32_t num_threads;          /* numThreads -> GPU shards (min with GPUs) */
  int32_t verbosity;            /* 1: Mallet's INFO lines on stderr         */
  int32_t reserved;
  int64_t seed;                 /* the Philox key (randomSeed, or the time-
                                   derived seed the Java side picked)       */
} ldaj_options;

/* Mallet's topicBits for numTopics: bitCount(topicMask), topicMask = K-1 for
 * a power of two, else highestOneBit(K)*2-1. */
int32_t ldaj_topic_bits(int32_t num_topics);

/* One GpuParallelTopicModel.estimate().
 *   doc_off[D+1], words[N]     the documents (FeatureSequence ids < V)
 *   z[N]                       in: topicSequence of every token (Mallet's
 *                              addInstances draws); out: after the sweeps
 *   alpha[K]                   in/out
 *   hyper[3]                   in/out: alphaSum, beta, betaSum
 *   sweep                      in/out: Philox sweep counter
 *   row_off[V+1]               typeTopicCounts row lengths as Mallet allocated
 *                              them (min(K, typeTotals[w]))
 *   rows[row_off[V]]           out: packed rows (count << topicBits | topic),
 *                              count-descending, trailing cells 0
 *   tokens_per_topic[K]        out
 *   ll_iter / ll_value [cap]   out: (iteration, LL/token) every 10 iterations;
 *                              *ll_n = how many (may exceed cap)
 * Status codes and lda_last_error-style text as lda_topic_model.h
 * (ldaj_last_error). */
lda_status ldaj_estimate(int32_t K, int32_t V, int64_t D, const int64_t* doc_off,
                         const int32_t* words, const ldaj_options* opt, int32_t* z, double* alpha,
                         double* hyper, uint32_t* sweep, const int64_t* row_off, int32_t* rows,
                         int32_t* tokens_per_topic, int32_t* ll_iter, double* ll_value,
                         int32_t ll_cap, int32_t* ll_n);

const char* ldaj_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LDA_JNI_CORE_H */
