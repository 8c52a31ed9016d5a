/*
 * estimate_harness.c — makes the native call of
 * cmu_gpu.GpuParallelTopicModel.estimate() (integration/java/...) from C,
 * with the same marshalling the Java method does, so the JNI path's native
 * half is compiled and GPU-tested in an image without a JDK.
 *
 *   estimate_harness IN OUT
 * IN  (little-endian): int32 K, V, D; int64 doc_off[D+1]; int32 words[N];
 *     int32 z[N] (Mallet's topicSequence); double alpha[K]; double hyper[3]
 *     (alphaSum, beta, betaSum); int64 sweep; int32 options[7]
 *     (numIterations, burninPeriod, optimizeInterval, saveSampleInterval,
 *     usingSymmetricAlpha, numThreads, verbosity); int64 seed
 * OUT: int32 z[N]; double alpha[K]; double hyper[3]; int64 sweep;
 *     int64 row_off[V+1]; int32 rows[row_off[V]]; int32 tokensPerTopic[K];
 *     int32 n_ll; int32 ll_iter[n_ll]; double ll_value[n_ll]
 * Exit status 0, or 2 with ldaj_last_error() on stderr.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../../integration/jni/lda_jni_core.h"

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
  if (argc != 3) {
    fprintf(stderr, "usage: %s IN OUT\n", argv[0]);
    return 1;
  }
  FILE* in = fopen(argv[1], "rb");
  if (!in) return 1;
  int32_t K, V, D;
  rd(in, &K, 4, 1);
  rd(in, &V, 4, 1);
  rd(in, &D, 4, 1);
  int64_t* doc_off = malloc(8 * (size_t)(D + 1));
  rd(in, doc_off, 8, (size_t)D + 1);
  const int64_t N = doc_off[D] - doc_off[0];
  int32_t* words = malloc(4 * (size_t)(N + 1));
  int32_t* z = malloc(4 * (size_t)(N + 1));
  rd(in, words, 4, (size_t)N);
  rd(in, z, 4, (size_t)N);
  double* alpha = malloc(8 * (size_t)K);
  double hyper[3];
  int64_t sweep64, seed;
  int32_t o[7];
  rd(in, alpha, 8, (size_t)K);
  rd(in, hyper, 8, 3);
  rd(in, &sweep64, 8, 1);
  rd(in, o, 4, 7);
  rd(in, &seed, 8, 1);
  fclose(in);

  /* GpuParallelTopicModel.estimate(): rows as Mallet's addInstances allocated
   * them (min(numTopics, typeTotals[type])), LL buffers for every 10th
   * iteration, the options array, the sweep counter field */
  int64_t* row_off = calloc((size_t)V + 1, 8);
  int64_t* totals = calloc((size_t)V, 8);
  for (int64_t i = 0; i < N; ++i) totals[words[i]]++;
  for (int32_t w = 0; w < V; ++w) row_off[w + 1] = row_off[w] + (totals[w] < K ? totals[w] : K);
  int32_t* rows = malloc(4 * (size_t)(row_off[V] + 1));
  int32_t* tpt = malloc(4 * (size_t)K);
  const int32_t cap = o[0] / 10 + 1;
  int32_t* ll_iter = malloc(4 * (size_t)cap);
  double* ll_value = malloc(8 * (size_t)cap);
  ldaj_options opt = {o[0], o[1], o[2], o[3], o[4], o[5], o[6], 0, seed};
  uint32_t sweep = (uint32_t)sweep64;
  int32_t n_ll = 0;
  lda_status st = ldaj_estimate(K, V, D, doc_off, words, &opt, z, alpha, hyper, &sweep, row_off,
                                rows, tpt, ll_iter, ll_value, cap, &n_ll);
  if (st != LDA_OK) {
    fprintf(stderr, "ldaj_estimate: %d %s\n", st, ldaj_last_error());
    return 2;
  }
  sweep64 = sweep;
  if (n_ll > cap) n_ll = cap;
  FILE* out = fopen(argv[2], "wb");
  if (!out) return 1;
  wr(out, z, 4, (size_t)N);
  wr(out, alpha, 8, (size_t)K);
  wr(out, hyper, 8, 3);
  wr(out, &sweep64, 8, 1);
  wr(out, row_off, 8, (size_t)V + 1);
  wr(out, rows, 4, (size_t)row_off[V]);
  wr(out, tpt, 4, (size_t)K);
  wr(out, &n_ll, 4, 1);
  wr(out, ll_iter, 4, (size_t)n_ll);
  wr(out, ll_value, 8, (size_t)n_ll);
  fclose(out);
  return 0;
}
