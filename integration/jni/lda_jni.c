/*
 * lda_jni.c — JNI glue for cmu_gpu.GpuParallelTopicModel over the C ABI in
 * include/lda_mi355x.h.  Build on a box with a JDK:
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -I../../include lda_jni.c -L../../ldagibbssampling_amd/lib -llda_mi355x \
 *       -Wl,-rpath,'$ORIGIN' -o liblda_mi355x_jni.so
 * Not compiled in the build image (no jni.h).  Errors become
 * java.lang.RuntimeException with lda_last_error().
 */
#include <jni.h>
#include <stdint.h>
#include <stdlib.h>

#include "lda_mi355x.h"

static int check(JNIEnv* env, lda_status s) {
  if (s == LDA_OK) return 0;
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  (*env)->ThrowNew(env, ex, lda_last_error());
  return 1;
}

JNIEXPORT jlong JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeCreate(
    JNIEnv* env, jclass cls, jint K, jint V, jlongArray docOff, jintArray words, jintArray z,
    jdoubleArray alpha, jdouble beta, jlong seed, jint device) {
  lda_config cfg = {0};
  jsize D = (*env)->GetArrayLength(env, docOff) - 1;
  jdouble* a = (*env)->GetDoubleArrayElements(env, alpha, NULL);
  jlong* off = (*env)->GetLongArrayElements(env, docOff, NULL);
  jint* w = (*env)->GetIntArrayElements(env, words, NULL);
  jint* zz = (*env)->GetIntArrayElements(env, z, NULL);
  cfg.num_topics = K;
  cfg.num_types = V;
  cfg.num_docs = D;
  cfg.alpha = a;
  cfg.beta = beta;
  cfg.seed = (uint64_t)seed;
  cfg.device = device;
  lda_ctx* ctx = NULL;
  lda_status s = lda_create(&ctx, &cfg, (const int64_t*)off, (const int32_t*)w, (const int32_t*)zz);
  (*env)->ReleaseIntArrayElements(env, z, zz, JNI_ABORT);
  (*env)->ReleaseIntArrayElements(env, words, w, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, docOff, off, JNI_ABORT);
  (*env)->ReleaseDoubleArrayElements(env, alpha, a, JNI_ABORT);
  if (check(env, s)) return 0;
  return (jlong)(intptr_t)ctx;
}

JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeSweep(JNIEnv* env, jclass cls,
                                                                        jlong ctx, jint n) {
  check(env, lda_sweep((lda_ctx*)(intptr_t)ctx, n));
}

JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeGetZ(JNIEnv* env, jclass cls,
                                                                       jlong ctx, jintArray z) {
  jint* p = (*env)->GetIntArrayElements(env, z, NULL);
  lda_status s = lda_get_z((lda_ctx*)(intptr_t)ctx, (int32_t*)p);
  (*env)->ReleaseIntArrayElements(env, z, p, 0);
  check(env, s);
}

JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeSetAlphaBeta(
    JNIEnv* env, jclass cls, jlong ctx, jdoubleArray alpha, jdouble beta) {
  jdouble* a = (*env)->GetDoubleArrayElements(env, alpha, NULL);
  lda_status s = lda_set_alpha_beta((lda_ctx*)(intptr_t)ctx, a, beta);
  (*env)->ReleaseDoubleArrayElements(env, alpha, a, JNI_ABORT);
  check(env, s);
}

JNIEXPORT jdouble JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeLogLikelihood(JNIEnv* env,
                                                                                   jclass cls,
                                                                                   jlong ctx) {
  double ll = 0.0;
  check(env, lda_log_likelihood((lda_ctx*)(intptr_t)ctx, &ll));
  return ll;
}

JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeMalletPacked(
    JNIEnv* env, jclass cls, jlong ctx, jintArray rows, jlongArray rowOff) {
  jlong* off = (*env)->GetLongArrayElements(env, rowOff, NULL);
  jint* r = rows ? (*env)->GetIntArrayElements(env, rows, NULL) : NULL;
  int32_t bits = 0;
  lda_status s = lda_to_mallet_packed((lda_ctx*)(intptr_t)ctx, (int32_t*)r, (int64_t*)off, &bits);
  if (r) (*env)->ReleaseIntArrayElements(env, rows, r, 0);
  (*env)->ReleaseLongArrayElements(env, rowOff, off, 0);
  check(env, s);
}

JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeGetTokensPerTopic(
    JNIEnv* env, jclass cls, jlong ctx, jintArray tpt) {
  jint* p = (*env)->GetIntArrayElements(env, tpt, NULL);
  lda_status s = lda_get_counts((lda_ctx*)(intptr_t)ctx, NULL, (int32_t*)p, NULL, NULL);
  (*env)->ReleaseIntArrayElements(env, tpt, p, 0);
  check(env, s);
}

/* alpha statistics: docLengthCounts[maxLen+1] and topicDocCounts flattened
 * [K*(maxLen+1)] are ADDED into (WorkerRunnable's collectAlphaStatistics) */
JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeDocTopicHistograms(
    JNIEnv* env, jclass cls, jlong ctx, jint maxLen, jintArray docLen, jintArray topicDoc) {
  jint* dl = (*env)->GetIntArrayElements(env, docLen, NULL);
  jint* td = (*env)->GetIntArrayElements(env, topicDoc, NULL);
  lda_status s = lda_doc_topic_histograms((lda_ctx*)(intptr_t)ctx, maxLen, (int32_t*)dl, (int32_t*)td);
  (*env)->ReleaseIntArrayElements(env, topicDoc, td, 0);
  (*env)->ReleaseIntArrayElements(env, docLen, dl, 0);
  check(env, s);
}

/* optimizeBeta's countHistogram[maxCount+1] (added into) */
JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeCountHistogram(
    JNIEnv* env, jclass cls, jlong ctx, jlong maxCount, jintArray hist) {
  jint* h = (*env)->GetIntArrayElements(env, hist, NULL);
  lda_status s = lda_count_histogram((lda_ctx*)(intptr_t)ctx, maxCount, (int32_t*)h);
  (*env)->ReleaseIntArrayElements(env, hist, h, 0);
  check(env, s);
}

JNIEXPORT void JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeDestroy(JNIEnv* env, jclass cls,
                                                                          jlong ctx) {
  lda_destroy((lda_ctx*)(intptr_t)ctx);
}
