/*
 * fake_env.c — TEST INFRASTRUCTURE: runs the JNI glue
 * (integration/jni/lda_jni.c, Java_cmu_1gpu_GpuParallelTopicModel_nativeEstimate)
 * through a fake JNIEnv, so its pinning, release modes and error paths execute
 * in an image without a JDK.  Built against tests/jni/stub/jni.h (the nine
 * JNIEnv functions the glue calls, restated from the JNI specification); the
 * fake's Java arrays behave as HotSpot's: Get<Type>ArrayElements returns a COPY
 * (isCopy = true), mode 0 copies back and frees, JNI_ABORT frees, JNI_COMMIT
 * copies back.
 *
 *   fake_env IN OUT             the call (input / output files as
 *                               tests/jni/estimate_harness.c) -> exit 0
 *   fake_env --fail-pin N IN    the N-th (1-based) Get<Type>ArrayElements
 *                               returns NULL with OutOfMemoryError pending
 *   fake_env --bad-k IN         K = 0: ldaj_estimate fails, RuntimeException
 * Every mode prints one line "pins=P releases=R aborts=A copies=C throws=T
 * pending=<class> ret=X" and checks itself: every pinned array is released
 * exactly once, never twice, and outputs are copied back only on success.
 * Exit 0 when the checks hold, 4 otherwise.
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../integration/jni/lda_jni_core.h"

JNIEXPORT jint JNICALL Java_cmu_1gpu_GpuParallelTopicModel_nativeEstimate(
    JNIEnv* env, jclass cls, jint K, jint V, jlongArray docOff, jintArray words, jintArray z,
    jdoubleArray alpha, jdoubleArray hyper, jlongArray sweep, jintArray options, jlong seed,
    jlongArray rowOff, jintArray rows, jintArray tokensPerTopic, jintArray llIter,
    jdoubleArray llValue);

struct _jobject {
  int is_class;
  const char* name;   /* class objects */
  size_t elem;        /* arrays */
  jsize len;
  void* data;         /* the Java array */
  void* copy;         /* the pinned copy handed out, or NULL */
  int pins, releases, copied_back, written_mode;
};

static int g_pin_calls, g_fail_at, g_throws, g_errors;
static const char* g_pending;
static char g_msg[600];
static struct _jobject g_class_rte = {1, "java/lang/RuntimeException", 0, 0, 0, 0, 0, 0, 0, -1};

static void bad(const char* what) {
  fprintf(stderr, "fake_env: %s\n", what);
  g_errors++;
}

static jclass FindClass(JNIEnv* env, const char* name) {
  (void)env;
  if (strcmp(name, g_class_rte.name) != 0) bad("FindClass of an unexpected class");
  return &g_class_rte;
}
static jint ThrowNew(JNIEnv* env, jclass c, const char* msg) {
  (void)env;
  if (g_pending) bad("ThrowNew with an exception already pending");
  g_throws++;
  g_pending = c->name;
  snprintf(g_msg, sizeof g_msg, "%s", msg ? msg : "");
  return 0;
}
static jsize GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  return a->len;
}
static void* get_elems(jarray a, size_t elem, jboolean* isCopy) {
  g_pin_calls++;
  if (a->elem != elem) bad("Get<Type>ArrayElements of the wrong element type");
  if (g_pending) bad("JNI call with an exception pending");
  if (g_fail_at && g_pin_calls == g_fail_at) {
    g_pending = "java/lang/OutOfMemoryError";
    return NULL;
  }
  if (a->copy) bad("array pinned twice");
  a->copy = malloc(elem * (size_t)(a->len ? a->len : 1));
  memcpy(a->copy, a->data, elem * (size_t)a->len);
  a->pins++;
  if (isCopy) *isCopy = JNI_TRUE;
  return a->copy;
}
static void release_elems(jarray a, void* p, jint mode) {
  if (!a->copy || p != a->copy) {
    bad("release of an array that is not pinned (or of another pointer)");
    return;
  }
  a->written_mode = mode;
  if (mode == 0 || mode == JNI_COMMIT) {
    memcpy(a->data, a->copy, a->elem * (size_t)a->len);
    a->copied_back++;
  }
  if (mode != JNI_COMMIT) {
    free(a->copy);
    a->copy = NULL;
    a->releases++;
  }
}
static jint* GetIntArrayElements(JNIEnv* env, jintArray a, jboolean* c) {
  (void)env;
  return (jint*)get_elems(a, sizeof(jint), c);
}
static jlong* GetLongArrayElements(JNIEnv* env, jlongArray a, jboolean* c) {
  (void)env;
  return (jlong*)get_elems(a, sizeof(jlong), c);
}
static jdouble* GetDoubleArrayElements(JNIEnv* env, jdoubleArray a, jboolean* c) {
  (void)env;
  return (jdouble*)get_elems(a, sizeof(jdouble), c);
}
static void ReleaseIntArrayElements(JNIEnv* env, jintArray a, jint* p, jint m) {
  (void)env;
  release_elems(a, p, m);
}
static void ReleaseLongArrayElements(JNIEnv* env, jlongArray a, jlong* p, jint m) {
  (void)env;
  release_elems(a, p, m);
}
static void ReleaseDoubleArrayElements(JNIEnv* env, jdoubleArray a, jdouble* p, jint m) {
  (void)env;
  release_elems(a, p, m);
}

static const struct JNINativeInterface_ g_table = {
    FindClass, ThrowNew, GetArrayLength, GetIntArrayElements, GetLongArrayElements, GetDoubleArrayElements,
    ReleaseIntArrayElements, ReleaseLongArrayElements, ReleaseDoubleArrayElements,
};

static struct _jobject* new_array(size_t elem, jsize len) {
  struct _jobject* a = calloc(1, sizeof *a);
  a->elem = elem;
  a->len = len;
  a->data = calloc(len ? (size_t)len : 1, elem);
  a->written_mode = -1;
  return a;
}

static void rd(FILE* f, void* p, size_t sz, size_t n) {
  if (n && fread(p, sz, n, f) != n) {
    fprintf(stderr, "short read\n");
    exit(3);
  }
}
static void wr(FILE* f, const void* p, size_t sz, size_t n) {
  if (n && fwrite(p, sz, n, f) != n) {
    fprintf(stderr, "short write\n");
    exit(3);
  }
}

int main(int argc, char** argv) {
  int a0 = 1, bad_k = 0;
  if (argc > 2 && strcmp(argv[1], "--fail-pin") == 0) {
    g_fail_at = atoi(argv[2]);
    a0 = 3;
  } else if (argc > 1 && strcmp(argv[1], "--bad-k") == 0) {
    bad_k = 1;
    a0 = 2;
  }
  const int run = !g_fail_at && !bad_k;
  if (argc != a0 + (run ? 2 : 1)) {
    fprintf(stderr, "usage: %s [--fail-pin N | --bad-k] IN [OUT]\n", argv[0]);
    return 1;
  }
  FILE* in = fopen(argv[a0], "rb");
  if (!in) return 1;
  int32_t K, V, D;
  rd(in, &K, 4, 1);
  rd(in, &V, 4, 1);
  rd(in, &D, 4, 1);
  /* GpuParallelTopicModel.estimate()'s arrays (integration/java/...) */
  jlongArray docOff = new_array(8, D + 1);
  rd(in, docOff->data, 8, (size_t)D + 1);
  const int64_t* off = docOff->data;
  const jsize N = (jsize)(off[D] - off[0]);
  jintArray words = new_array(4, N), z = new_array(4, N);
  rd(in, words->data, 4, (size_t)N);
  rd(in, z->data, 4, (size_t)N);
  jdoubleArray alpha = new_array(8, K), hyper = new_array(8, 3);
  jlongArray sweep = new_array(8, 1);
  jintArray options = new_array(4, 7);
  int64_t seed;
  rd(in, alpha->data, 8, (size_t)K);
  rd(in, hyper->data, 8, 3);
  rd(in, sweep->data, 8, 1);
  rd(in, options->data, 4, 7);
  rd(in, &seed, 8, 1);
  fclose(in);
  jlongArray rowOff = new_array(8, V + 1);
  int64_t* ro = rowOff->data;
  int64_t* totals = calloc((size_t)V, 8);
  for (jsize i = 0; i < N; ++i) totals[((int32_t*)words->data)[i]]++;
  for (int32_t w = 0; w < V; ++w) ro[w + 1] = ro[w] + (totals[w] < K ? totals[w] : K);
  jintArray rows = new_array(4, (jsize)ro[V]), tpt = new_array(4, K);
  const int32_t cap = ((int32_t*)options->data)[0] / 10 + 1;
  jintArray llIter = new_array(4, cap);
  jdoubleArray llValue = new_array(8, cap);
  int32_t* z0 = malloc(4 * (size_t)(N ? N : 1));
  memcpy(z0, z->data, 4 * (size_t)N);

  JNIEnv env = &g_table;
  const jint ret = Java_cmu_1gpu_GpuParallelTopicModel_nativeEstimate(
      &env, NULL, bad_k ? 0 : K, V, docOff, words, z, alpha, hyper, sweep, options, (jlong)seed, rowOff, rows, tpt,
      llIter, llValue);

  /* every array pinned was released exactly once; outputs copied back only on success */
  struct _jobject* all[] = {docOff, words, z, alpha, hyper, sweep, options, rowOff, rows, tpt, llIter, llValue};
  const int is_out[] = {0, 0, 1, 1, 1, 1, 0, 0, 1, 1, 1, 1};
  int pins = 0, releases = 0, aborts = 0, copies = 0;
  for (int i = 0; i < 12; ++i) {
    struct _jobject* a = all[i];
    pins += a->pins;
    releases += a->releases;
    copies += a->copied_back;
    if (a->copy) bad("an array is still pinned");
    if (a->pins != a->releases) bad("pins and releases differ");
    if (a->pins > 1) bad("an array was pinned more than once");
    if (a->releases && a->written_mode == JNI_ABORT) aborts++;
    const int expect_copy = run && is_out[i];
    if (a->copied_back != expect_copy) bad(expect_copy ? "an output was not copied back" : "an array was copied back");
  }
  if (run) {
    if (g_pending || g_throws) bad("exception on the success path");
    if (pins != 12) bad("not every array was pinned");
  } else if (g_fail_at) {
    if (ret != 0 || !g_pending || strcmp(g_pending, "java/lang/OutOfMemoryError") != 0 || g_throws)
      bad("a failed pin must leave only the JVM's OutOfMemoryError pending and return 0");
    if (memcmp(z0, z->data, 4 * (size_t)N) != 0) bad("z changed after a failed pin");
  } else {
    if (ret != 0 || g_throws != 1 || !g_pending || strcmp(g_pending, "java/lang/RuntimeException") != 0 || !g_msg[0])
      bad("an ldaj_estimate error must throw one RuntimeException with a message");
    if (memcmp(z0, z->data, 4 * (size_t)N) != 0) bad("z changed after an error");
  }
  printf("pins=%d releases=%d aborts=%d copies=%d throws=%d pending=%s ret=%d msg=%s\n", pins, releases, aborts,
         copies, g_throws, g_pending ? g_pending : "none", (int)ret, g_msg);
  if (run && !g_errors) {
    FILE* out = fopen(argv[a0 + 1], "wb");
    if (!out) return 1;
    int32_t n_ll = ret < cap ? ret : cap;
    wr(out, z->data, 4, (size_t)N);
    wr(out, alpha->data, 8, (size_t)K);
    wr(out, hyper->data, 8, 3);
    wr(out, sweep->data, 8, 1);
    wr(out, ro, 8, (size_t)V + 1);
    wr(out, rows->data, 4, (size_t)ro[V]);
    wr(out, tpt->data, 4, (size_t)K);
    wr(out, &n_ll, 4, 1);
    wr(out, llIter->data, 4, (size_t)n_ll);
    wr(out, llValue->data, 8, (size_t)n_ll);
    fclose(out);
  }
  return g_errors ? 4 : 0;
}
