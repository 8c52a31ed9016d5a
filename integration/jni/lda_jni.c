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
 *
 * Failure behaviour (tests/jni/fake_env.c runs every path through a fake
 * JNIEnv):
 *   - a Get<Type>ArrayElements that returns NULL leaves the JVM's
 *     OutOfMemoryError pending: every array pinned so far is released with
 *     JNI_ABORT and the call returns 0 without a second exception;
 *   - an ldaj_estimate error releases every array with JNI_ABORT and throws
 *     java.lang.RuntimeException carrying ldaj_last_error().  On a JVM that
 *     hands out copies (isCopy == JNI_TRUE, HotSpot's usual behaviour) the
 *     Java arrays keep their values; on one that pins them in place
 *     (isCopy == JNI_FALSE, which the JNI spec allows) ldaj_estimate may
 *     already have written z, alpha, the packed rows and tokensPerTopic, and
 *     JNI_ABORT cannot undo that: after the exception those arrays are
 *     indeterminate and the model must be rebuilt (Mallet's own estimate()
 *     gives no stronger guarantee on an exception);
 *   - on success the inputs (docOff, words, options, rowOff) are released with
 *     JNI_ABORT and the outputs with mode 0 (copied back).
 */
#include <jni.h>
#include <stdint.h>

#include "lda_jni_core.h"

static void throw_status(JNIEnv* env) {
  jclass ex = (*env)->FindClass(env, "java/lang/RuntimeException");
  if (ex) (*env)->ThrowNew(env, ex, ldaj_last_error());
}

enum { P_OFF, P_WORDS, P_Z, P_ALPHA, P_HYPER, P_SWEEP, P_ROWOFF, P_ROWS, P_TPT, P_LLI, P_LLV, P_COUNT };

typedef struct {
  jarray arr;
  void* ptr;
  char kind;   /* 'I', 'J', 'D' */
  char out;    /* 1: written back on success */
} pin_t;

static void* pin(JNIEnv* env, pin_t* p) {
  switch (p->kind) {
    case 'I': p->ptr = (*env)->GetIntArrayElements(env, (jintArray)p->arr, NULL); break;
    case 'J': p->ptr = (*env)->GetLongArrayElements(env, (jlongArray)p->arr, NULL); break;
    default: p->ptr = (*env)->GetDoubleArrayElements(env, (jdoubleArray)p->arr, NULL); break;
  }
  return p->ptr;
}

static void unpin(JNIEnv* env, pin_t* p, int ok) {
  if (!p->ptr) return;
  const jint mode = (ok && p->out) ? 0 : JNI_ABORT;
  switch (p->kind) {
    case 'I': (*env)->ReleaseIntArrayElements(env, (jintArray)p->arr, (jint*)p->ptr, mode); break;
    case 'J': (*env)->ReleaseLongArrayElements(env, (jlongArray)p->arr, (jlong*)p->ptr, mode); break;
    default: (*env)->ReleaseDoubleArrayElements(env, (jdoubleArray)p->arr, (jdouble*)p->ptr, mode); break;
  }
  p->ptr = NULL;
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
  if (!o) return 0;   /* OutOfMemoryError pending */
  ldaj_options opt = {o[0], o[1], o[2], o[3], o[4], o[5], o[6], 0, (int64_t)seed};
  (*env)->ReleaseIntArrayElements(env, options, o, JNI_ABORT);

  pin_t p[P_COUNT] = {
      {docOff, NULL, 'J', 0}, {words, NULL, 'I', 0},        {z, NULL, 'I', 1},
      {alpha, NULL, 'D', 1},  {hyper, NULL, 'D', 1},        {sweep, NULL, 'J', 1},
      {rowOff, NULL, 'J', 0}, {rows, NULL, 'I', 1},         {tokensPerTopic, NULL, 'I', 1},
      {llIter, NULL, 'I', 1}, {llValue, NULL, 'D', 1},
  };
  for (int i = 0; i < P_COUNT; ++i)
    if (!pin(env, &p[i])) {
      /* the JVM threw OutOfMemoryError: release what is pinned, unchanged */
      for (int j = i - 1; j >= 0; --j) unpin(env, &p[j], 0);
      return 0;
    }

  jlong* sw = (jlong*)p[P_SWEEP].ptr;
  uint32_t s32 = (uint32_t)sw[0];
  int32_t n_ll = 0;
  lda_status st = ldaj_estimate(K, V, D, (const int64_t*)p[P_OFF].ptr, (const int32_t*)p[P_WORDS].ptr, &opt,
                                (int32_t*)p[P_Z].ptr, (double*)p[P_ALPHA].ptr, (double*)p[P_HYPER].ptr, &s32,
                                (const int64_t*)p[P_ROWOFF].ptr, (int32_t*)p[P_ROWS].ptr,
                                (int32_t*)p[P_TPT].ptr, (int32_t*)p[P_LLI].ptr, (double*)p[P_LLV].ptr, cap, &n_ll);
  const int ok = st == LDA_OK;
  if (ok) sw[0] = (jlong)s32;
  for (int j = P_COUNT - 1; j >= 0; --j) unpin(env, &p[j], ok);
  if (!ok) {
    throw_status(env);
    return 0;
  }
  return n_ll;
}
