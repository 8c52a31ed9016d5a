/*
 * lda_jni.c — JNI glue for cmu_gpu.GpuParallelTopicModel: pins the Java
 * arrays and calls ldaj_estimate (lda_jni_core.c), which is plain C over
 * include/lda_topic_model.h and is compiled and GPU-tested in the build image
 * (tests/jni/estimate_harness.c).  Only this file needs jni.h.  Build on a box
 * with a JDK (integration/jni/Makefile, target `jni`):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux \
 *       -I../../include lda_jni.c lda_jni_core.c \
 *       -L../../ldagibbssampling_amd/lib -llda_topic_model -llda_mi355x \
 *       -Wl,-rpath,'$ORIGIN' -o liblda_mi355x_jni.so
 * Errors become java.lang.RuntimeException carrying ldaj_last_error().
 */
#include <jni.h>
#include <stdint.h>

#include "lda_jni_core.h"

static void throw_status(JNIEnv* env) {
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  (*env)->ThrowNew(env, ex, ldaj_last_error());
}

/* options[7] = numIterations, burninPeriod, optimizeInterval,
 *              saveSampleInterval, usingSymmetricAlpha, numThreads, verbosity
 * hyper[3]   = alphaSum, beta, betaSum (in/out)
 * sweep[1]   = Philox sweep counter (in/out)
 * returns the number of (iteration, LL/token) pairs written into llIter/llValue */
JNIEXPORT jint JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeEstimate(
    JNIEnv* env, jclass cls, jint K, jint V, jlongArray docOff, jintArray words, jintArray z,
    jdoubleArray alpha, jdoubleArray hyper, jlongArray sweep, jintArray options, jlong seed,
    jlongArray rowOff, jintArray rows, jintArray tokensPerTopic, jintArray llIter,
    jdoubleArray llValue) {
  (void)cls;
  const jsize D = (*env)->GetArrayLength(env, docOff) - 1;
  const jsize cap = (*env)->GetArrayLength(env, llIter);
  jint* o = (*env)->GetIntArrayElements(env, options, NULL);
  ldaj_options opt = {o[0], o[1], o[2], o[3], o[4], o[5], o[6], 0, (int64_t)seed};
  (*env)->ReleaseIntArrayElements(env, options, o, JNI_ABORT);

  jlong* off = (*env)->GetLongArrayElements(env, docOff, NULL);
  jint* w = (*env)->GetIntArrayElements(env, words, NULL);
  jint* zz = (*env)->GetIntArrayElements(env, z, NULL);
  jdouble* a = (*env)->GetDoubleArrayElements(env, alpha, NULL);
  jdouble* h = (*env)->GetDoubleArrayElements(env, hyper, NULL);
  jlong* sw = (*env)->GetLongArrayElements(env, sweep, NULL);
  jlong* ro = (*env)->GetLongArrayElements(env, rowOff, NULL);
  jint* r = (*env)->GetIntArrayElements(env, rows, NULL);
  jint* tpt = (*env)->GetIntArrayElements(env, tokensPerTopic, NULL);
  jint* li = (*env)->GetIntArrayElements(env, llIter, NULL);
  jdouble* lv = (*env)->GetDoubleArrayElements(env, llValue, NULL);

  uint32_t s32 = (uint32_t)sw[0];
  int32_t n_ll = 0;
  lda_status st = ldaj_estimate(K, V, D, (const int64_t*)off, (const int32_t*)w, &opt, (int32_t*)zz,
                                a, h, &s32, (const int64_t*)ro, (int32_t*)r, (int32_t*)tpt,
                                (int32_t*)li, lv, cap, &n_ll);
  sw[0] = (jlong)s32;

  (*env)->ReleaseDoubleArrayElements(env, llValue, lv, 0);
  (*env)->ReleaseIntArrayElements(env, llIter, li, 0);
  (*env)->ReleaseIntArrayElements(env, tokensPerTopic, tpt, 0);
  (*env)->ReleaseIntArrayElements(env, rows, r, 0);
  (*env)->ReleaseLongArrayElements(env, rowOff, ro, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, sweep, sw, 0);
  (*env)->ReleaseDoubleArrayElements(env, hyper, h, 0);
  (*env)->ReleaseDoubleArrayElements(env, alpha, a, 0);
  (*env)->ReleaseIntArrayElements(env, z, zz, 0);
  (*env)->ReleaseIntArrayElements(env, words, w, JNI_ABORT);
  (*env)->ReleaseLongArrayElements(env, docOff, off, JNI_ABORT);
  if (st != LDA_OK) {
    throw_status(env);
    return 0;
  }
  return n_ll;
}
