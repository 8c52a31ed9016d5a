/*
 * lda_jni_core.c — see lda_jni_core.h.  Plain C over include/lda_topic_model.h.
 */
#include "lda_jni_core.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static _Thread_local char g_err[512];

const char* ldaj_last_error(void) { return g_err; }

static lda_status fail(lda_status s, const char* what, const char* detail) {
  snprintf(g_err, sizeof g_err, "%s%s%s", what, detail ? ": " : "", detail ? detail : "");
  return s;
}

#define TM(call)                                                  \
  do {                                                            \
    lda_status s_ = (call);                                       \
    if (s_ != LDA_OK) {                                           \
      st = fail(s_, #call, ldatm_last_error());                   \
      goto done;                                                  \
    }                                                             \
  } while (0)

int32_t ldaj_topic_bits(int32_t K) {
  int32_t mask;
  if ((K & (K - 1)) == 0) {
    mask = K - 1;
  } else {
    int32_t hb = 1;
    while (hb * 2 <= K) hb *= 2;
    mask = hb * 2 - 1;
  }
  return __builtin_popcount((unsigned)mask);
}

static int cmp_desc(const void* a, const void* b) {
  const int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
  return (x < y) - (x > y);
}

lda_status ldaj_estimate(int32_t K, int32_t V, int64_t D, const int64_t* doc_off,
                         const int32_t* words, const ldaj_options* opt, int32_t* z, double* alpha,
                         double* hyper, uint32_t* sweep, const int64_t* row_off, int32_t* rows,
                         int32_t* tokens_per_topic, int32_t* ll_iter, double* ll_value,
                         int32_t ll_cap, int32_t* ll_n) {
  if (K < 1 || V < 1 || D < 0 || !doc_off || !opt || !alpha || !hyper || !sweep || !row_off ||
      !tokens_per_topic || !ll_n || (ll_cap > 0 && (!ll_iter || !ll_value)))
    return fail(LDA_ERR_INVALID_ARG, "ldaj_estimate", "bad argument");
  const int64_t N = doc_off[D] - doc_off[0];
  if (N > 0 && (!words || !z)) return fail(LDA_ERR_INVALID_ARG, "ldaj_estimate", "null tokens");
  if (row_off[V] > 0 && !rows) return fail(LDA_ERR_INVALID_ARG, "ldaj_estimate", "null rows");
  const int32_t bits = ldaj_topic_bits(K);
  lda_status st = LDA_OK;
  g_err[0] = '\0';
  ldatm* m = NULL;
  int32_t* nw = NULL;
  int32_t* cell = NULL;
  int32_t n_trace = 0;
  *ll_n = 0;

  TM(ldatm_create(&m, K, hyper[0], hyper[1]));
  TM(ldatm_set_alphabet(m, V, NULL));
  TM(ldatm_add_instances(m, D, doc_off, words, NULL));
  TM(ldatm_set_topics(m, N, z));                         /* Mallet's own random topics */
  TM(ldatm_set_hyper(m, alpha, hyper[0], hyper[1]));
  TM(ldatm_set_random_seed(m, opt->seed));
  TM(ldatm_set_num_threads(m, opt->num_threads > 0 ? opt->num_threads : 1));
  TM(ldatm_set_num_iterations(m, opt->num_iterations));
  TM(ldatm_set_burnin_period(m, opt->burnin_period));
  TM(ldatm_set_optimize_interval(m, opt->optimize_interval));
  TM(ldatm_set_save_sample_interval(m, opt->save_sample_interval > 0 ? opt->save_sample_interval : 10));
  TM(ldatm_set_symmetric_alpha(m, opt->symmetric_alpha));
  TM(ldatm_set_topic_display(m, 0, 0));
  TM(ldatm_set_verbosity(m, opt->verbosity));
  TM(ldatm_set_sweep(m, *sweep));                        /* continue the random stream */
  TM(ldatm_estimate(m));

  /* write-back: what Mallet's fields hold after estimate() */
  TM(ldatm_get_z(m, z));
  {
    double a_sum = 0.0, beta = 0.0;
    TM(ldatm_get_hyper(m, alpha, &a_sum, &beta));
    hyper[0] = a_sum;
    hyper[1] = beta;
    hyper[2] = beta * (double)V;
  }
  TM(ldatm_get_sweep(m, sweep));
  TM(ldatm_get_ll_trace(m, ll_iter, ll_value, ll_cap, &n_trace));
  *ll_n = n_trace;
  nw = (int32_t*)malloc(sizeof(int32_t) * (size_t)V * (size_t)K);
  cell = (int32_t*)malloc(sizeof(int32_t) * (size_t)K);
  if (!nw || !cell) {
    st = fail(LDA_ERR_OUT_OF_MEMORY, "ldaj_estimate", "host allocation");
    goto done;
  }
  TM(ldatm_get_counts(m, nw, tokens_per_topic));
  for (int32_t w = 0; w < V; ++w) {
    int32_t n = 0;
    for (int32_t k = 0; k < K; ++k) {
      const int32_t c = nw[(size_t)w * K + k];
      if (c > 0) {
        if ((int64_t)c >= ((int64_t)1 << (31 - bits))) {
          st = fail(LDA_ERR_UNSUPPORTED, "ldaj_estimate", "count does not fit Mallet's packed cell");
          goto done;
        }
        cell[n++] = (c << bits) | k;
      }
    }
    const int64_t len = row_off[w + 1] - row_off[w];
    if (n > len) {
      st = fail(LDA_ERR_INVALID_ARG, "ldaj_estimate", "a typeTopicCounts row is shorter than its nonzero topics");
      goto done;
    }
    qsort(cell, (size_t)n, sizeof(int32_t), cmp_desc);
    for (int64_t i = 0; i < len; ++i) rows[row_off[w] + i] = i < n ? cell[i] : 0;
  }

done:
  free(nw);
  free(cell);
  if (m) ldatm_destroy(m);
  return st;
}
