#define _GNU_SOURCE
/*
 * lda_oracle.c — CPU restatements of the collapsed-Gibbs LDA hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see lda_oracle.h for the contract and the parity
 * status: the Mallet restatement is "parity unpinned" against Mallet 2.0.7,
 * which cannot be built or run in this image; cpu_exact is the bit-exact
 * oracle for the HIP sampler and is pinned by the committed golden fixtures).
 *
 * Compile with -ffp-contract=off: every fp32 fused multiply-add below is an
 * explicit fmaf(), exactly where the HIP kernel issues v_fma_f32, and no other
 * operation may be contracted.
 */
#include "lda_oracle.h"

#include <math.h>
#include <pthread.h>
#include <sched.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

/* ======================================================================== */
/* Philox4x32-10 — Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as  */
/* easy as 1, 2, 3", SC'11; constants and round structure as in Random123's */
/* philox.h.  Pinned by tests/test_oracle.py against the published KATs.    */
/* ======================================================================== */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += PHILOX_W0;
      k1 += PHILOX_W1;
    }
    uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
    uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    uint32_t n0 = hi1 ^ c1 ^ k0;
    uint32_t n1 = lo1;
    uint32_t n2 = hi0 ^ c3 ^ k1;
    uint32_t n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t orc_draw(uint64_t seed, uint64_t gtok, uint32_t c2, uint32_t c3) {
  uint32_t ctr[4] = {(uint32_t)gtok, (uint32_t)(gtok >> 32), c2, c3};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  uint32_t out[4];
  orc_philox4x32_10(ctr, key, out);
  return out[0];
}

/* all four words of the token's Philox block (the large-K draw uses x1, x2) */
void orc_draw4(uint64_t seed, uint64_t gtok, uint32_t c2, uint32_t c3, uint32_t out[4]) {
  uint32_t ctr[4] = {(uint32_t)gtok, (uint32_t)(gtok >> 32), c2, c3};
  uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  orc_philox4x32_10(ctr, key, out);
}

float orc_u01(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

/* Philox stream ids (counter word 3). */
#define STREAM_SAMPLE 0u
#define STREAM_INIT 1u
#define STREAM_INFER 2u

/* ======================================================================== */
/* java.util.Random: 48-bit LCG (JDK spec), base of cc.mallet.util.Randoms.  */
/* ======================================================================== */
#define JR_MULT 0x5DEECE66DULL
#define JR_MASK ((1ULL << 48) - 1)

void orc_jrandom_seed(orc_jrandom* r, int64_t seed) { r->s = ((uint64_t)seed ^ JR_MULT) & JR_MASK; }

static inline int32_t jr_next(orc_jrandom* r, int bits) {
  r->s = (r->s * JR_MULT + 0xBULL) & JR_MASK;
  return (int32_t)(int64_t)(r->s >> (48 - bits));
}

int32_t orc_jrandom_next_int(orc_jrandom* r) { return jr_next(r, 32); }

int32_t orc_jrandom_next_int_n(orc_jrandom* r, int32_t n) {
  if ((n & -n) == n) return (int32_t)(((int64_t)n * (int64_t)jr_next(r, 31)) >> 31);
  int32_t bits, val;
  do {
    bits = jr_next(r, 31);
    val = bits % n;
  } while (bits - val + (n - 1) < 0);
  return val;
}

double orc_jrandom_next_double(orc_jrandom* r) {
  int64_t hi = (int64_t)jr_next(r, 26);
  int64_t lo = (int64_t)jr_next(r, 27);
  return (double)((hi << 27) + lo) * 0x1p-53;
}

/* ======================================================================== */
/* cc.mallet.types.Dirichlet.logGammaStirling [M]                            */
/* ======================================================================== */
double orc_log_gamma_stirling(double z) {
  const double HALF_LOG_TWO_PI = log(2.0 * M_PI) / 2.0;
  int shift = 0;
  while (z < 2) {
    z++;
    shift++;
  }
  double result = HALF_LOG_TWO_PI + (z - 0.5) * log(z) - z + 1 / (12 * z) - 1 / (360 * z * z * z) +
                  1 / (1260 * z * z * z * z * z);
  while (shift > 0) {
    shift--;
    z--;
    result -= log(z);
  }
  return result;
}

/* ======================================================================== */
/* cc.mallet.types.Dirichlet: digamma, learnParameters,                      */
/* learnSymmetricConcentration [M] (Minka's fixed-point iterations)          */
/* ======================================================================== */
double orc_digamma(double x) {
  /* psi(x) = psi(x + n) - sum_{j<n} 1/(x + j); asymptotic series above 9.5 */
  const double EULER = 0.5772156649015328606065121;
  if (x < 1e-6) return -EULER - 1.0 / x;
  double acc = 0.0;
  for (; x < 9.5; x += 1.0) acc -= 1.0 / x;
  const double r = 1.0 / x, r2 = r * r;
  const double series =
      1.0 / 12 - r2 * (1.0 / 120 - r2 * (1.0 / 252 - r2 * (1.0 / 240 - r2 * (1.0 / 132 -
      r2 * (691.0 / 32760 - r2 * (1.0 / 12))))));
  return acc + (log(x) - 0.5 * r - r2 * series);
}

double orc_learn_parameters(double* a, int32_t K, const int32_t* hist, const int32_t* lens,
                            int32_t L, double shape, double scale, int32_t iters) {
  const int64_t W = (int64_t)L + 1;
  double A = 0.0;
  int64_t* top = (int64_t*)malloc(sizeof(int64_t) * (K > 0 ? K : 1));
  for (int32_t k = 0; k < K; ++k) {
    A += a[k];
    top[k] = -1;
    for (int64_t i = W - 1; i >= 0; --i)
      if (hist[k * W + i] > 0) {
        top[k] = i;
        break;
      }
  }
  for (int32_t it = 0; it < iters; ++it) {
    double den = 0.0, d = 0.0;
    for (int64_t n = 1; n < W; ++n) {
      d += 1.0 / (A + (double)(n - 1));
      den += lens[n] * d;
    }
    den -= 1.0 / scale;
    A = 0.0;
    for (int32_t k = 0; k < K; ++k) {
      const double ak = a[k];
      double num = 0.0;
      d = 0.0;
      for (int64_t i = 1; i <= top[k]; ++i) {
        d += 1.0 / (ak + (double)(i - 1));   /* not (ak + i) - 1: cancels for ak < 1.1e-16 */
        num += hist[k * W + i] * d;
      }
      a[k] = ak * (num + shape) / den;
      if (a[k] < 1e-300) a[k] = 1e-300;     /* a dead topic must not underflow to 0 */
      A += a[k];
    }
  }
  free(top);
  return A;
}

/* observation lengths as a DENSE histogram lens[0..max_len] (Mallet's form) */
double orc_learn_symmetric_concentration(const int32_t* counts, int64_t max_count,
                                         const int32_t* lens, int64_t max_len, int32_t dims,
                                         double value) {
  int64_t top = 0;
  for (int64_t c = max_count; c > 0; --c)
    if (counts[c] > 0) {
      top = c;
      break;
    }
  for (int it = 0; it < 200; ++it) {
    const double p = value / dims;
    double num = 0.0, d = 0.0;
    /* the numerator over the non-zero counts, with Mallet's denominator rule
     * (digamma difference across gaps > 20, term by term otherwise): equal
     * to Mallet's literal loop for histograms without such gaps */
    const double pbase = orc_digamma(p);
    int64_t prevc = 0;
    for (int64_t c = 1; c <= top; ++c) {
      if (counts[c] <= 0) continue;
      if (c - prevc > 20)
        d = orc_digamma(p + (double)c) - pbase;
      else
        for (int64_t i = prevc + 1; i <= c; ++i) d += 1.0 / (p + (double)(i - 1));
      num += counts[c] * d;
      prevc = c;
    }
    const double psi0 = orc_digamma(value);
    double den = 0.0;
    int64_t last = 0;
    d = 0.0;
    for (int64_t n = 0; n <= max_len; ++n) {
      if (lens[n] <= 0) continue;
      if (n - last > 20)
        d = orc_digamma(value + n) - psi0;
      else
        for (int64_t i = last; i < n; ++i) d += 1.0 / (value + i);
      den += d * lens[n];
      last = n;
    }
    value = p * num / den;
  }
  return value;
}

/* ======================================================================== */
/* cpu_exact                                                                */
/* ======================================================================== */
struct orc_exact {
  int32_t K, Kp, C, V;
  int64_t D, N;
  int64_t* doc_off;
  int32_t* words;
  int32_t* z;
  int32_t* nw;    /* V*Kp snapshot */
  int32_t* nwsum; /* Kp */
  int32_t* delta; /* V*Kp + Kp */
  double* alpha;  /* K */
  double beta;
  float* alpha_f; /* Kp (0 in the padding) */
  float beta_f, vbeta_f;
  float* inv;    /* Kp: 1/(nwsum + V*beta), 0 in the padding */
  float* inv_m1; /* Kp: 1/(nwsum - 1 + V*beta) */
  /* the large-K draw's tables (exact_draw_big; lda_kernels.hip k_big_tables) */
  float* ainv;    /* Kp: alpha_f * inv */
  float* ainv_m1; /* Kp: alpha_f * inv_m1 (0 for a topic with no tokens) */
  uint32_t *bF, *bFm1, *bG, *bGm1; /* Kp: big_fix of inv, inv_m1, ainv, ainv_m1 */
  uint64_t* bpfx; /* Kp: inclusive prefix of bG */
  int32_t bS;     /* fixed-point exponent */
  uint64_t bS0;   /* sum of bG */
  float bsig, bsig_hi; /* beta * 2^-S, beta * 2^(32-S) */
  double isig;         /* 2^S / beta */
  uint64_t seed;
  int64_t token_base;
  uint32_t sweep;
  int kind; /* 0 = dense draw, 1 = sparse (SparseLDA-split) draw */
  int half; /* dense, K <= 128: 1 = the half-wave variant's draw, 2 = the quarter-wave one */
};

/* The large-K draw's fixed-point doc part (ldagibbssampling_amd/csrc/
 * lda_kernels.hip: k_big_tables).  m = the largest of inv_k, ainv_k and, for
 * topics holding tokens, inv_m1_k and ainv_m1_k; S = 31 - e with m = f 2^e,
 * f in [0.5, 1), so big_fix(x) = (uint32) ldexpf(x, S) < 2^31 for every table
 * value (a power-of-two scaling is exact; the conversion truncates). */
static uint32_t big_fix(float x, int S) { return (uint32_t)ldexpf(x, S); }

static void exact_big_tables(orc_exact* s) {
  float m = 0.0f;
  for (int k = 0; k < s->Kp; ++k) {
    const int live = k < s->K && s->nwsum[k] >= 1;
    s->ainv[k] = s->alpha_f[k] * s->inv[k];
    s->ainv_m1[k] = live ? s->alpha_f[k] * s->inv_m1[k] : 0.0f;
    const float im1 = live ? s->inv_m1[k] : 0.0f;
    m = fmaxf(m, fmaxf(fmaxf(s->inv[k], s->ainv[k]), fmaxf(im1, s->ainv_m1[k])));
  }
  int e = 0;
  (void)frexpf(m, &e);
  s->bS = m > 0.0f ? 31 - e : 0;
  uint64_t acc = 0;
  for (int k = 0; k < s->Kp; ++k) {
    const int live = k < s->K && s->nwsum[k] >= 1;
    s->bF[k] = big_fix(s->inv[k], s->bS);
    s->bFm1[k] = live ? big_fix(s->inv_m1[k], s->bS) : 0u;
    s->bG[k] = big_fix(s->ainv[k], s->bS);
    s->bGm1[k] = big_fix(s->ainv_m1[k], s->bS);
    acc += s->bG[k];
    s->bpfx[k] = acc;
  }
  s->bS0 = acc;
  s->bsig = ldexpf(s->beta_f, -s->bS);
  s->bsig_hi = ldexpf(s->beta_f, 32 - s->bS);
  s->isig = ldexp(1.0, s->bS) / (double)s->beta_f;
}

static void exact_prepare_topics(orc_exact* s) {
  for (int k = 0; k < s->Kp; ++k) {
    if (k < s->K) {
      s->alpha_f[k] = (float)s->alpha[k];
      s->inv[k] = 1.0f / ((float)s->nwsum[k] + s->vbeta_f);
      s->inv_m1[k] = 1.0f / ((float)(s->nwsum[k] - 1) + s->vbeta_f);
    } else {
      s->alpha_f[k] = 0.0f;
      s->inv[k] = 0.0f;
      s->inv_m1[k] = 0.0f;
    }
  }
  exact_big_tables(s);
}

orc_exact* orc_exact_create(int32_t K, int32_t V, int64_t D, const int64_t* doc_off,
                            const int32_t* words, const int32_t* z_init, const double* alpha,
                            double beta, uint64_t seed, int64_t token_base) {
  orc_exact* s = (orc_exact*)calloc(1, sizeof(orc_exact));
  s->K = K;
  /* 64 x the next power of two >= ceil(K/64): every C has a kernel
   * instantiation (ldagibbssampling_amd/csrc/lda_capi.cpp:pad_topics). */
  s->Kp = 64;
  while (s->Kp < K) s->Kp *= 2;
  s->C = s->Kp / 64;
  /* dense K <= 128: the library's default kernel is the quarter-wave one
   * (lda_capi.cpp: LDA_DENSE_HALF unset), so its draw is the default here */
  s->half = 2;
  s->V = V;
  s->D = D;
  s->N = doc_off[D] - doc_off[0];
  s->doc_off = (int64_t*)malloc(sizeof(int64_t) * (D + 1));
  for (int64_t d = 0; d <= D; ++d) s->doc_off[d] = doc_off[d] - doc_off[0];
  s->words = (int32_t*)malloc(sizeof(int32_t) * (s->N ? s->N : 1));
  s->z = (int32_t*)malloc(sizeof(int32_t) * (s->N ? s->N : 1));
  memcpy(s->words, words, sizeof(int32_t) * s->N);
  s->nw = (int32_t*)calloc((size_t)V * s->Kp, sizeof(int32_t));
  s->nwsum = (int32_t*)calloc(s->Kp, sizeof(int32_t));
  s->delta = (int32_t*)calloc((size_t)V * s->Kp + s->Kp, sizeof(int32_t));
  s->alpha = (double*)malloc(sizeof(double) * K);
  memcpy(s->alpha, alpha, sizeof(double) * K);
  s->beta = beta;
  s->alpha_f = (float*)calloc(s->Kp, sizeof(float));
  s->inv = (float*)calloc(s->Kp, sizeof(float));
  s->inv_m1 = (float*)calloc(s->Kp, sizeof(float));
  s->ainv = (float*)calloc(s->Kp, sizeof(float));
  s->ainv_m1 = (float*)calloc(s->Kp, sizeof(float));
  s->bF = (uint32_t*)calloc(s->Kp, sizeof(uint32_t));
  s->bFm1 = (uint32_t*)calloc(s->Kp, sizeof(uint32_t));
  s->bG = (uint32_t*)calloc(s->Kp, sizeof(uint32_t));
  s->bGm1 = (uint32_t*)calloc(s->Kp, sizeof(uint32_t));
  s->bpfx = (uint64_t*)calloc(s->Kp, sizeof(uint64_t));
  s->beta_f = (float)beta;
  s->vbeta_f = (float)((double)V * beta);
  s->seed = seed;
  s->token_base = token_base;
  s->sweep = 0;
  for (int64_t i = 0; i < s->N; ++i) {
    if (z_init) {
      s->z[i] = z_init[i];
    } else {
      uint32_t x = orc_draw(seed, (uint64_t)(token_base + i), 0u, STREAM_INIT);
      s->z[i] = (int32_t)(((uint64_t)x * (uint64_t)K) >> 32);
    }
  }
  /* local counts become the pending delta; the first apply (after an
   * all-reduce when sharded) turns them into the global snapshot. */
  int32_t* dsum = s->delta + (size_t)V * s->Kp;
  for (int64_t i = 0; i < s->N; ++i) {
    s->delta[(size_t)s->words[i] * s->Kp + s->z[i]] += 1;
    dsum[s->z[i]] += 1;
  }
  exact_prepare_topics(s);
  return s;
}

void orc_exact_destroy(orc_exact* s) {
  if (!s) return;
  free(s->doc_off); free(s->words); free(s->z); free(s->nw); free(s->nwsum); free(s->delta);
  free(s->alpha); free(s->alpha_f); free(s->inv); free(s->inv_m1);
  free(s->ainv); free(s->ainv_m1); free(s->bF); free(s->bFm1); free(s->bG); free(s->bGm1);
  free(s->bpfx);
  free(s);
}

int32_t orc_exact_kpad(const orc_exact* s) { return s->Kp; }
int32_t* orc_exact_delta(orc_exact* s) { return s->delta; }
void orc_exact_set_sweep(orc_exact* s, uint32_t sweep) { s->sweep = sweep; }
void orc_exact_set_kind(orc_exact* s, int kind) { s->kind = kind; }
void orc_exact_set_half(orc_exact* s, int half) { s->half = half; }
uint32_t orc_exact_get_sweep(const orc_exact* s) { return s->sweep; }

void orc_exact_apply(orc_exact* s) {
  size_t nv = (size_t)s->V * s->Kp;
  for (size_t i = 0; i < nv; ++i) {
    s->nw[i] += s->delta[i];
    s->delta[i] = 0;
  }
  for (int k = 0; k < s->Kp; ++k) {
    s->nwsum[k] += s->delta[nv + k];
    s->delta[nv + k] = 0;
  }
  exact_prepare_topics(s);
}

/* Replace the snapshot by an external global one (nw[V*K] unpadded, nwsum[K]):
 * checks a slice of a larger corpus against the GPU's state of that corpus. */
void orc_exact_load_snapshot(orc_exact* s, const int32_t* nw, const int32_t* nwsum) {
  memset(s->nw, 0, sizeof(int32_t) * (size_t)s->V * s->Kp);
  memset(s->nwsum, 0, sizeof(int32_t) * s->Kp);
  memset(s->delta, 0, sizeof(int32_t) * ((size_t)s->V * s->Kp + s->Kp));
  for (int w = 0; w < s->V; ++w)
    memcpy(s->nw + (size_t)w * s->Kp, nw + (size_t)w * s->K, sizeof(int32_t) * s->K);
  memcpy(s->nwsum, nwsum, sizeof(int32_t) * s->K);
  exact_prepare_topics(s);
}

void orc_exact_set_alpha_beta(orc_exact* s, const double* alpha, double beta) {
  memcpy(s->alpha, alpha, sizeof(double) * s->K);
  s->beta = beta;
  s->beta_f = (float)beta;
  s->vbeta_f = (float)((double)s->V * beta);
  exact_prepare_topics(s);
}

/* The wavefront inclusive scan of the kernel (DPP): row_shr 1,2,4,8 inside
 * 16-lane rows (out-of-row sources read 0), then row_bcast:15 into rows 1 and
 * 3, then row_bcast:31 into rows 2 and 3.  ldagibbssampling_amd/csrc/
 * lda_kernels.hip: wave_incl_scan(). */
static void wave_scan_emulate(float x[64]) {
  float y[64];
  for (int d = 1; d <= 8; d <<= 1) {
    for (int l = 0; l < 64; ++l) y[l] = ((l & 15) >= d) ? x[l - d] : 0.0f;
    for (int l = 0; l < 64; ++l) x[l] = y[l] + x[l];
  }
  for (int l = 0; l < 64; ++l) {
    int row = l >> 4;
    y[l] = (row == 1 || row == 3) ? x[16 * row - 1] : 0.0f;
  }
  for (int l = 0; l < 64; ++l) x[l] = x[l] + y[l];
  for (int l = 0; l < 64; ++l) y[l] = (l >= 32) ? x[31] : 0.0f;
  for (int l = 0; l < 64; ++l) x[l] = x[l] + y[l];
}

/* One categorical draw over the Kp padded topics.  nwrow = the snapshot row
 * of the token's word; nd = live doc counts with the token already removed;
 * zo = the token's old topic (-1: frozen, no self-correction). */
static int exact_draw(const orc_exact* s, const int32_t* nwrow, const int32_t* nd, int zo,
                      float u, float* S /* scratch Kp */) {
  const int C = s->C, K = s->K;
  float t[64];
  for (int l = 0; l < 64; ++l) {
    float acc = 0.0f;
    for (int j = 0; j < C; ++j) {
      int k = l * C + j;
      int32_t c = nwrow[k];
      float iv = s->inv[k];
      if (k == zo) {
        c -= 1;
        iv = s->inv_m1[k];
      }
      float b = ((float)c + s->beta_f) * iv;
      float a = (float)nd[k] + s->alpha_f[k];
      acc = fmaf(a, b, acc);
      S[k] = acc;
    }
    t[l] = acc;
  }
  wave_scan_emulate(t);
  float total = t[63];
  float thr = u * total;
  const int last_lane = (K - 1) / C;
  int lstar = last_lane;
  for (int l = 0; l <= last_lane; ++l) {
    if (t[l] > thr) {
      lstar = l;
      break;
    }
  }
  float E = lstar > 0 ? t[lstar - 1] : 0.0f;
  int cnt = 0;
  for (int j = 0; j < C; ++j) cnt += (E + S[lstar * C + j] <= thr) ? 1 : 0;
  int jsel;
  if (cnt < C) {
    jsel = cnt;
  } else {
    jsel = (lstar < last_lane) ? C - 1 : (K - 1) % C;
  }
  return lstar * C + jsel;
}

/* The half-wave dense draw (K <= 128; lda_kernels.hip: k_sample_half): two
 * documents per wavefront, so one token's topics spread over the 32 lanes of
 * a half, CH = 1, 2, 4 topics per lane for K <= 32, 64, 128.  The per-lane
 * serial fma prefix is exact_draw's; the scan is the half's 32-lane one
 * (row_shr 1,2,4,8 inside 16-lane rows, then row_bcast:15 into its second
 * row), thr = u * T_31, and the lane / element selection follow exact_draw. */
static int half_topics_per_lane(int K) { return K <= 32 ? 1 : (K <= 64 ? 2 : 4); }

static int exact_draw_half(const orc_exact* s, const int32_t* nwrow, const int32_t* nd, int zo,
                           float u, float* S) {
  const int K = s->K, CH = half_topics_per_lane(K);
  float t[32], y[32];
  for (int l = 0; l < 32; ++l) {
    float acc = 0.0f;
    for (int j = 0; j < CH; ++j) {
      const int k = l * CH + j;
      int32_t c = nwrow[k];
      float iv = s->inv[k];
      if (k == zo) {
        c -= 1;
        iv = s->inv_m1[k];
      }
      const float b = ((float)c + s->beta_f) * iv;
      const float a = (float)nd[k] + s->alpha_f[k];
      acc = fmaf(a, b, acc);
      S[k] = acc;
    }
    t[l] = acc;
  }
  for (int d = 1; d <= 8; d <<= 1) {
    for (int l = 0; l < 32; ++l) y[l] = ((l & 15) >= d) ? t[l - d] : 0.0f;
    for (int l = 0; l < 32; ++l) t[l] = y[l] + t[l];
  }
  for (int l = 16; l < 32; ++l) t[l] = t[l] + t[15];
  const float thr = u * t[31];
  const int last_lane = (K - 1) / CH;
  int lstar = last_lane;
  for (int l = 0; l <= last_lane; ++l)
    if (t[l] > thr) {
      lstar = l;
      break;
    }
  const float E = lstar > 0 ? t[lstar - 1] : 0.0f;
  int cnt = 0;
  for (int j = 0; j < CH; ++j) cnt += (E + S[lstar * CH + j] <= thr) ? 1 : 0;
  const int lim = lstar < last_lane ? CH - 1 : (K - 1) % CH;
  return lstar * CH + (cnt < lim ? cnt : lim);
}

/* The quarter-wave dense draw (K <= 128; lda_kernels.hip: k_sample_quarter,
 * LDA_DENSE_HALF=2): four documents per wavefront, one token's topics over the
 * 16 lanes of one DPP row, CH = 1, 2, 4, 8 topics per lane for K <= 16, 32, 64,
 * 128.  The per-lane serial fma prefix is exact_draw's; T = the row's
 * inclusive scan (row_shr 1,2,4,8); thr = u * T_15; l* = min(#{l : T_l <=
 * thr}, last lane) (the first lane with T > thr: T is monotone); E, the count
 * and the clamp as exact_draw.  The document factor a_k is the kernel's running
 * fp32 value af[k] (exact_sample_docs): float(nd_k) + alpha_k when the
 * document starts, then -1.0f when a token leaves topic k and +1.0f when one
 * joins it, in token order (LDS float atomics on the GPU). */
static int quarter_topics_per_lane(int K) { return K <= 16 ? 1 : (K <= 32 ? 2 : (K <= 64 ? 4 : 8)); }

static int exact_draw_quarter(const orc_exact* s, const int32_t* nwrow, const float* af, int zo,
                              float u, float* S) {
  const int K = s->K, CH = quarter_topics_per_lane(K);
  float t[16], y[16];
  for (int l = 0; l < 16; ++l) {
    float acc = 0.0f;
    for (int j = 0; j < CH; ++j) {
      const int k = l * CH + j;
      int32_t c = nwrow[k];
      float iv = s->inv[k];
      if (k == zo) {
        c -= 1;
        iv = s->inv_m1[k];
      }
      const float b = ((float)c + s->beta_f) * iv;
      acc = fmaf(af[k], b, acc);
      S[k] = acc;
    }
    t[l] = acc;
  }
  for (int d = 1; d <= 8; d <<= 1) {
    for (int l = 0; l < 16; ++l) y[l] = l >= d ? t[l - d] : 0.0f;
    for (int l = 0; l < 16; ++l) t[l] = y[l] + t[l];
  }
  const float thr = u * t[15];
  const int last_lane = (K - 1) / CH;
  int cle = 0;
  for (int l = 0; l < 16; ++l) cle += (t[l] <= thr) ? 1 : 0;
  const int lstar = cle < last_lane ? cle : last_lane;
  const float E = lstar > 0 ? t[lstar - 1] : 0.0f;
  int cnt = 0;
  for (int j = 0; j < CH; ++j) cnt += (E + S[lstar * CH + j] <= thr) ? 1 : 0;
  const int lim = lstar < last_lane ? CH - 1 : (K - 1) % CH;
  return lstar * CH + (cnt < lim ? cnt : lim);
}

/* The sparse draw (kind 1, ldagibbssampling_amd/csrc/lda_kernels.hip:
 * k_sample_sparse / k_sample_sparse_big).  The same p_k =
 * (nd_k + a_k)(nw_k + b) inv_k is split as
 *   coef_k = (float(nd_k) + alpha_k) * (k == zo ? inv_m1_k : inv_k)
 *   B_e    = coef[t_e] * float(c_e - [t_e == zo])   over the word's nonzero
 *            entries e (topic ascending), lane l holding e = l, l+64, ...
 *   A_k    = coef_k * beta  (all topics, lane l owning [l*C, l*C+C))
 * B: per-lane serial sums (add), DPP scan; A: per-lane grouped fma chains
 * (lane_partial_grouped), DPP scan; thr = u * (sumB + sumA); B first. */
/* Dense doc part of the sparse draw, per lane: topics [l*C, l*C+C) in groups
 * of GS = min(C, 16); G_g = serial fma(coef, beta) over group g,
 * TA_l = ((G_0 + G_1) + G_2) + ...; the prefix at element j of group g is
 * x_j = (G_0 + ... + G_{g-1}) + s_{g,j}  (s = serial fma inside the group).
 * For C <= 16 (one group) this is the plain serial fma chain. */
/* Doc-part partials of the sparse draw.  C <= 16: one serial fma chain of
 * coef*beta per lane.  C >= 32 (k_sample_sparse_big): groups of 16 topics,
 * each the Hillis-Steele inclusive scan of p_j = coef_j*beta across a 16-lane
 * DPP row (row_shr 1,2,4,8; out-of-row sources add 0); x[] = the in-group
 * prefix, G = x[15]; the lane partial is ((G0 + G1) + G2) + ... */
static float group_rowscan16(const float* coef16, float beta, float x[16]) {
  for (int j = 0; j < 16; ++j) x[j] = coef16[j] * beta;
  for (int d = 1; d < 16; d <<= 1) {
    float y[16];
    for (int j = 0; j < 16; ++j) y[j] = j >= d ? x[j - d] : 0.0f;
    for (int j = 0; j < 16; ++j) x[j] = x[j] + y[j];
  }
  return x[15];
}

static float lane_partial_grouped(const float* coef_lane, int C, float beta, float* G) {
  if (C <= 16) {
    float a = 0.0f;
    for (int j = 0; j < C; ++j) a = fmaf(coef_lane[j], beta, a);
    G[0] = a;
    return a;
  }
  float tot = 0.0f, x[16];
  for (int g = 0; g < C / 16; ++g) {
    G[g] = group_rowscan16(coef_lane + 16 * g, beta, x);
    tot = g == 0 ? G[g] : tot + G[g];
  }
  return tot;
}

static int exact_draw_sparse(const orc_exact* s, const int32_t* nwrow, const int32_t* nd, int zo,
                             float u, float* coef, int32_t* et, int32_t* ec) {
  const int C = s->C, K = s->K, Kp = s->Kp;
  for (int k = 0; k < Kp; ++k)
    coef[k] = ((float)nd[k] + s->alpha_f[k]) * (k == zo ? s->inv_m1[k] : s->inv[k]);
  int n = 0;
  for (int k = 0; k < K; ++k)
    if (nwrow[k] > 0) {
      et[n] = k;
      ec[n] = nwrow[k] - (k == zo ? 1 : 0);
      n++;
    }
  float TB[64], TA[64], G[4];
  for (int l = 0; l < 64; ++l) {
    float acc = 0.0f;
    for (int e = l; e < n; e += 64) acc = acc + coef[et[e]] * (float)ec[e];
    TB[l] = acc;
    TA[l] = lane_partial_grouped(coef + l * C, C, s->beta_f, G);
  }
  wave_scan_emulate(TB);
  wave_scan_emulate(TA);
  const float sumB = TB[63], sumA = TA[63];
  const float thr = u * (sumB + sumA);
  if (thr < sumB) {
    const int nl = n < 64 ? n : 64;
    int lstar = nl - 1;
    for (int l = 0; l < nl; ++l)
      if (TB[l] > thr) {
        lstar = l;
        break;
      }
    const float E = lstar > 0 ? TB[lstar - 1] : 0.0f;
    float acc = 0.0f;
    int cnt = 0, nr = 0;
    for (int e = lstar; e < n; e += 64) {
      acc = acc + coef[et[e]] * (float)ec[e];
      cnt += (E + acc <= thr) ? 1 : 0;
      nr++;
    }
    const int r = cnt < nr ? cnt : nr - 1;
    return et[lstar + 64 * r];
  }
  const float thr2 = thr - sumB;
  const int last_lane = (K - 1) / C;
  int lstar = last_lane;
  for (int l = 0; l <= last_lane; ++l)
    if (TA[l] > thr2) {
      lstar = l;
      break;
    }
  const float E = lstar > 0 ? TA[lstar - 1] : 0.0f;
  int cnt = 0;
  if (C <= 16) {
    float a = 0.0f;
    for (int j = 0; j < C; ++j) {
      a = fmaf(coef[lstar * C + j], s->beta_f, a);
      cnt += (E + a <= thr2) ? 1 : 0;
    }
  } else {
    float P = 0.0f, x[16];
    for (int g = 0; g < C / 16; ++g) {
      const float Gg = group_rowscan16(coef + lstar * C + 16 * g, s->beta_f, x);
      for (int j = 0; j < 16; ++j) cnt += (E + (g == 0 ? x[j] : P + x[j]) <= thr2) ? 1 : 0;
      P = g == 0 ? Gg : P + Gg;
    }
  }
  const int jsel = cnt < C ? cnt : ((lstar < last_lane) ? C - 1 : (K - 1) % C);
  return lstar * C + jsel;
}

/* The large-K sparse draw (kind 1, C >= 32; lda_kernels.hip: k_sample_big,
 * round 5).  The same p_k = (nd_k + a_k)(nw_k + b) inv_k, split as
 *   B (word part) over the word's nonzero entries e (topic ascending, lane l
 *     holding e = l, l+64, ...), WITHOUT the own-token correction:
 *       coef_t = fmaf(float(nd_t), inv_t, ainv_t), ainv = alpha * inv
 *       acc_l  = fmaf(float(c_e), coef_{t_e}, acc_l)   (per-lane running sum)
 *     TB = the kernel's DPP wave scan of acc_l (wave_scan_emulate).
 *   A (doc part, beta * sum_k (nd_k + a_k) inv'_k) exactly, in fixed point:
 *       A_fx = sum_k nd_k F'_k + sum_k G'_k  (uint64; F = big_fix(inv),
 *       G = big_fix(ainv); ' = the _m1 values at the token's own topic zo)
 *       A_f  = fmaf(float(A_fx >> 32), beta 2^(32-S), float((uint32) A_fx) * beta 2^-S)
 *   thr = u0 * (sumB + A_f).
 * Selection (big_select): B first: the first lane with TB > thr, then the
 * count of its running sums <= thr - E; else A: tfx = floor(double(thr -
 * sumB) * isig), first the alpha part (prefix of G', topic ascending), then
 * the document part (prefix of nd F', topic ascending); K-1 when none.
 * The own token: B holds its entry as x = c * coef_zo where the exact weight
 * is O = (c - 1) * fmaf(nd_zo, inv_m1_zo, ainv_m1_zo) <= x.  A draw that lands
 * on it keeps zo when u1 * w < O (w = the entry's width in its lane's running
 * sums); otherwise the draw is repeated once over the same sums with the
 * entry's width replaced by O (thr2 = u2 * T', mapped around the entry), which
 * makes the result exactly the corrected distribution. */
typedef struct {
  int n;               /* word entries */
  const int32_t *et, *ec;
  const float* acc_e;  /* acc_e[e]: lane (e & 63)'s running sum after entry e */
  float TB[64];
  float sumB, A_f;
  uint64_t As;         /* the alpha part of A_fx */
  int64_t dG;          /* G'_zo - G_zo (0 when frozen) */
  int zo;              /* -1 when frozen */
} big_draw;

static int big_select(const orc_exact* s, const big_draw* d, const int32_t* nd, float thr, int* entry) {
  *entry = -1;
  if (thr < d->sumB) {
    const int nl = d->n < 64 ? d->n : 64;
    int lstar = nl - 1;
    for (int l = 0; l < nl; ++l)
      if (d->TB[l] > thr) {
        lstar = l;
        break;
      }
    const float E = lstar > 0 ? d->TB[lstar - 1] : 0.0f;
    const float thrE = thr - E;
    const int nr = (d->n - lstar + 63) / 64;
    int cnt = 0;
    for (int q = 0; q < nr; ++q) cnt += (d->acc_e[lstar + 64 * q] <= thrE) ? 1 : 0;
    *entry = lstar + 64 * (cnt < nr ? cnt : nr - 1);
    return d->et[*entry];
  }
  const float t2 = thr - d->sumB;
  const uint64_t tfx = (uint64_t)((double)t2 * s->isig);
  if (tfx < d->As) {
    for (int k = 0; k < s->K; ++k) {
      const int64_t v = (int64_t)s->bpfx[k] + (d->zo >= 0 && k >= d->zo ? d->dG : 0);
      if ((uint64_t)v > tfx) return k;
    }
    return s->K - 1;
  }
  const uint64_t tr = tfx - d->As;
  uint64_t acc = 0;
  for (int k = 0; k < s->K; ++k) {
    acc += (uint64_t)nd[k] * (k == d->zo ? s->bFm1[k] : s->bF[k]);
    if (acc > tr) return k;
  }
  return s->K - 1;
}

static int exact_draw_big(const orc_exact* s, const int32_t* nwrow, const int32_t* nd, int zo,
                          const uint32_t x[4], int32_t* et, int32_t* ec, float* acc_e) {
  const int K = s->K;
  big_draw d;
  d.n = 0;
  for (int k = 0; k < K; ++k)
    if (nwrow[k] > 0) {
      et[d.n] = k;
      ec[d.n] = nwrow[k];
      d.n++;
    }
  for (int l = 0; l < 64; ++l) {
    float acc = 0.0f;
    for (int e = l; e < d.n; e += 64) {
      const int t = et[e];
      acc = fmaf((float)ec[e], fmaf((float)nd[t], s->inv[t], s->ainv[t]), acc);
      acc_e[e] = acc;
    }
    d.TB[l] = acc;
  }
  wave_scan_emulate(d.TB);
  d.sumB = d.TB[63];
  uint64_t R = 0;
  for (int k = 0; k < s->Kp; ++k) R += (uint64_t)nd[k] * s->bF[k];
  int64_t dF = 0;
  d.dG = 0;
  if (zo >= 0) {
    dF = (int64_t)nd[zo] * ((int64_t)s->bFm1[zo] - (int64_t)s->bF[zo]);
    d.dG = (int64_t)s->bGm1[zo] - (int64_t)s->bG[zo];
  }
  d.zo = zo;
  d.As = (uint64_t)((int64_t)s->bS0 + d.dG);
  const uint64_t Afx = (uint64_t)((int64_t)(d.As + R) + dF);
  /* fp32: beta 2^-S (hi 2^32 + lo); hi < 2^16 is exact */
  d.A_f = fmaf((float)(uint32_t)(Afx >> 32), s->bsig_hi, (float)(uint32_t)Afx * s->bsig);
  d.et = et;
  d.ec = ec;
  d.acc_e = acc_e;
  const float T = d.sumB + d.A_f;
  int entry;
  const int kn = big_select(s, &d, nd, orc_u01(x[0]) * T, &entry);
  if (zo < 0 || entry < 0 || kn != zo) return kn;
  /* the own entry */
  const float hi = acc_e[entry], lo = entry >= 64 ? acc_e[entry - 64] : 0.0f;
  const float w = hi - lo;
  const int32_t cm1 = ec[entry] > 0 ? ec[entry] - 1 : 0;
  const float O = (float)cm1 * fmaf((float)nd[zo], s->inv_m1[zo], s->ainv_m1[zo]);
  if (orc_u01(x[1]) * w < O) return zo;
  const int l = entry & 63;
  const float s_lo = (l > 0 ? d.TB[l - 1] : 0.0f) + lo;
  const float Tp = ((d.sumB - w) + O) + d.A_f;
  const float thr2 = orc_u01(x[2]) * Tp;
  if (thr2 < s_lo) return big_select(s, &d, nd, thr2, &entry);
  if (thr2 < s_lo + O) return zo;
  return big_select(s, &d, nd, (thr2 - O) + w, &entry);
}

/* Test hook: one large-K draw for word w with document counts nd (the token
 * already removed), old topic zo (-1: frozen) and Philox words x[0..2]
 * (tests/test_oracle.py checks its distribution against the exact
 * conditional). */
int orc_exact_big_draw(const orc_exact* s, int32_t w, const int32_t* nd, int32_t zo, const uint32_t* x) {
  int32_t* et = (int32_t*)malloc(sizeof(int32_t) * s->Kp);
  int32_t* ec = (int32_t*)malloc(sizeof(int32_t) * s->Kp);
  float* acc_e = (float*)malloc(sizeof(float) * s->Kp);
  const int kn = exact_draw_big(s, s->nw + (size_t)w * s->Kp, nd, zo, x, et, ec, acc_e);
  free(et);
  free(ec);
  free(acc_e);
  return kn;
}

/* Sample the docs [d0, d1) of a token stream against the snapshot.  frozen:
 * no self-correction (inference).  The snapshot is read-only and nd is per
 * document, so disjoint document blocks are independent; the count changes
 * are derived afterwards from the old and new z (exact_sample_stream). */
static void exact_sample_docs(const orc_exact* s, const int64_t* doc_off, const int32_t* words,
                              int32_t* z, int64_t d0, int64_t d1, int frozen, uint32_t c2,
                              uint32_t c3, int64_t token_base) {
  int32_t* nd = (int32_t*)calloc(s->Kp, sizeof(int32_t));
  float* S = (float*)malloc(sizeof(float) * s->Kp);
  int32_t* et = (int32_t*)malloc(sizeof(int32_t) * s->Kp);
  int32_t* ec = (int32_t*)malloc(sizeof(int32_t) * s->Kp);
  float* af = (float*)malloc(sizeof(float) * s->Kp);
  float* acc_e = (float*)malloc(sizeof(float) * s->Kp);
  const int quarter = s->kind == 0 && s->half == 2 && s->Kp <= 128;
  const int big = s->kind == 1 && s->C >= 32;
  for (int64_t d = d0; d < d1; ++d) {
    memset(nd, 0, sizeof(int32_t) * s->Kp);
    for (int64_t i = doc_off[d]; i < doc_off[d + 1]; ++i) nd[z[i]]++;
    /* the quarter-wave kernel's running document factors (exact_draw_quarter) */
    for (int k = 0; k < s->Kp; ++k) af[k] = (float)nd[k] + s->alpha_f[k];
    for (int64_t i = doc_off[d]; i < doc_off[d + 1]; ++i) {
      int w = words[i];
      int zo = z[i];
      uint32_t x[4];
      orc_draw4(s->seed, (uint64_t)(token_base + i), c2, c3, x);
      float u = orc_u01(x[0]);
      nd[zo]--;
      af[zo] -= 1.0f;
      int kn = big ? exact_draw_big(s, s->nw + (size_t)w * s->Kp, nd, frozen ? -1 : zo, x, et, ec, acc_e)
               : s->kind == 1
                   ? exact_draw_sparse(s, s->nw + (size_t)w * s->Kp, nd, frozen ? -1 : zo, u, S, et, ec)
                   : quarter
                         ? exact_draw_quarter(s, s->nw + (size_t)w * s->Kp, af, frozen ? -1 : zo, u, S)
                   : (s->half == 1 && s->Kp <= 128)
                         ? exact_draw_half(s, s->nw + (size_t)w * s->Kp, nd, frozen ? -1 : zo, u, S)
                         : exact_draw(s, s->nw + (size_t)w * s->Kp, nd, frozen ? -1 : zo, u, S);
      nd[kn]++;
      af[kn] += 1.0f;
      z[i] = kn;
    }
  }
  free(af);
  free(acc_e);
  free(nd);
  free(S);
  free(et);
  free(ec);
}

/* Worker threads over contiguous document blocks (ORACLE_THREADS, default
 * min(16, online CPUs)): the result does not depend on the split. */
typedef struct {
  const orc_exact* s;
  const int64_t* doc_off;
  const int32_t* words;
  int32_t* z;
  int64_t d0, d1;
  int frozen;
  uint32_t c2, c3;
  int64_t token_base;
} exact_job;

static void* exact_job_run(void* arg) {
  exact_job* j = (exact_job*)arg;
  exact_sample_docs(j->s, j->doc_off, j->words, j->z, j->d0, j->d1, j->frozen, j->c2, j->c3,
                    j->token_base);
  return NULL;
}

static int oracle_threads(void) {
  const char* e = getenv("ORACLE_THREADS");
  long t = e ? atol(e) : sysconf(_SC_NPROCESSORS_ONLN);
  if (t < 1) t = 1;
  if (t > 16) t = 16;
  return (int)t;
}

static void exact_sample_stream(const orc_exact* s, const int64_t* doc_off, const int32_t* words,
                                int32_t* z, int64_t D, int frozen, uint32_t c2, uint32_t c3,
                                int64_t token_base, int32_t* delta) {
  const int64_t N = doc_off[D] - doc_off[0];
  int32_t* zold = NULL;
  if (delta) {
    zold = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
    memcpy(zold, z + doc_off[0], sizeof(int32_t) * N);
  }
  int T = oracle_threads();
  if ((int64_t)T > D) T = (int)(D > 0 ? D : 1);
  if (T <= 1 || N < 4096) {
    exact_sample_docs(s, doc_off, words, z, 0, D, frozen, c2, c3, token_base);
  } else {
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * T);
    exact_job* jobs = (exact_job*)malloc(sizeof(exact_job) * T);
    int64_t d = 0;
    for (int t = 0; t < T; ++t) {
      /* token-balanced cut: the first document starting at or after t*N/T */
      const int64_t target = doc_off[0] + N * (t + 1) / T;
      int64_t e = d;
      while (e < D && doc_off[e] < target) ++e;
      if (t == T - 1) e = D;
      exact_job j = {s, doc_off, words, z, d, e, frozen, c2, c3, token_base};
      jobs[t] = j;
      d = e;
    }
    for (int t = 0; t < T; ++t) pthread_create(&th[t], NULL, exact_job_run, &jobs[t]);
    for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
    free(th);
    free(jobs);
  }
  if (delta) {
    int32_t* dsum = delta + (size_t)s->V * s->Kp;
    for (int64_t i = 0; i < N; ++i) {
      const int zo = zold[i], kn = z[doc_off[0] + i];
      if (kn != zo) {
        const size_t row = (size_t)words[doc_off[0] + i] * s->Kp;
        delta[row + zo] -= 1;
        delta[row + kn] += 1;
        dsum[zo] -= 1;
        dsum[kn] += 1;
      }
    }
    free(zold);
  }
}

void orc_exact_sample(orc_exact* s, int frozen) {
  exact_sample_stream(s, s->doc_off, s->words, s->z, s->D, frozen, s->sweep, STREAM_SAMPLE,
                      s->token_base, frozen ? NULL : s->delta);
  s->sweep++;
}

/* Documents [d0, d1) of the current sweep only (the sweep counter is not
 * advanced; orc_exact_end_sweep does that): a split sweep's part, restated
 * for the tests of the exchange-overlapped driver (lda_sample_part). */
void orc_exact_sample_docs(orc_exact* s, int64_t d0, int64_t d1) {
  if (d0 < 0) d0 = 0;
  if (d1 > s->D) d1 = s->D;
  if (d1 <= d0) return;
  exact_sample_stream(s, s->doc_off + d0, s->words, s->z, d1 - d0, 0, s->sweep, STREAM_SAMPLE,
                      s->token_base, s->delta);
}

void orc_exact_end_sweep(orc_exact* s) { s->sweep++; }

void orc_exact_get_z(const orc_exact* s, int32_t* z) { memcpy(z, s->z, sizeof(int32_t) * s->N); }

void orc_exact_get_counts(const orc_exact* s, int32_t* nw, int32_t* nwsum, int32_t* nd,
                          int32_t* ndsum) {
  if (nw)
    for (int w = 0; w < s->V; ++w)
      for (int k = 0; k < s->K; ++k) nw[(size_t)w * s->K + k] = s->nw[(size_t)w * s->Kp + k];
  if (nwsum)
    for (int k = 0; k < s->K; ++k) nwsum[k] = s->nwsum[k];
  if (nd) {
    memset(nd, 0, sizeof(int32_t) * (size_t)s->D * s->K);
    for (int64_t d = 0; d < s->D; ++d)
      for (int64_t i = s->doc_off[d]; i < s->doc_off[d + 1]; ++i) nd[(size_t)d * s->K + s->z[i]]++;
  }
  if (ndsum)
    for (int64_t d = 0; d < s->D; ++d) ndsum[d] = (int32_t)(s->doc_off[d + 1] - s->doc_off[d]);
}

/* ParallelTopicModel.modelLogLikelihood() [M], restated over dense counts,
 * split into the document part (this shard's docs, incl. D*logG(alphaSum))
 * and the word part (global counts). */
static void mallet_ll_dense_parts(int K, int V, int Kstride, const double* alpha, double beta,
                                  int64_t D, const int64_t* doc_off, const int32_t* z,
                                  const int32_t* nw, const int32_t* nwsum, double* doc_part,
                                  double* word_part) {
  double alpha_sum = 0.0;
  for (int k = 0; k < K; ++k) alpha_sum += alpha[k];
  double ll = 0.0;
  double* topic_lg = (double*)malloc(sizeof(double) * K);
  int32_t* counts = (int32_t*)calloc(K, sizeof(int32_t));
  for (int k = 0; k < K; ++k) topic_lg[k] = orc_log_gamma_stirling(alpha[k]);
  for (int64_t d = 0; d < D; ++d) {
    for (int64_t i = doc_off[d]; i < doc_off[d + 1]; ++i) counts[z[i]]++;
    for (int k = 0; k < K; ++k)
      if (counts[k] > 0) ll += orc_log_gamma_stirling(alpha[k] + counts[k]) - topic_lg[k];
    ll -= orc_log_gamma_stirling(alpha_sum + (double)(doc_off[d + 1] - doc_off[d]));
    memset(counts, 0, sizeof(int32_t) * K);
  }
  ll += (double)D * orc_log_gamma_stirling(alpha_sum);
  *doc_part = ll;
  ll = 0.0;
  int64_t nonzero = 0;
  for (int w = 0; w < V; ++w)
    for (int k = 0; k < K; ++k) {
      int32_t c = nw[(size_t)w * Kstride + k];
      if (c > 0) {
        nonzero++;
        ll += orc_log_gamma_stirling(beta + c);
      }
    }
  for (int k = 0; k < K; ++k) ll -= orc_log_gamma_stirling(beta * V + nwsum[k]);
  ll += orc_log_gamma_stirling(beta * V) * K;
  ll -= orc_log_gamma_stirling(beta) * (double)nonzero;
  *word_part = ll;
  free(topic_lg);
  free(counts);
}

static double mallet_ll_dense(int K, int V, int Kstride, const double* alpha, double beta,
                              int64_t D, const int64_t* doc_off, const int32_t* z,
                              const int32_t* nw, const int32_t* nwsum) {
  double a, b;
  mallet_ll_dense_parts(K, V, Kstride, alpha, beta, D, doc_off, z, nw, nwsum, &a, &b);
  return a + b;
}

void orc_exact_log_likelihood_parts(const orc_exact* s, double* doc_part, double* word_part) {
  mallet_ll_dense_parts(s->K, s->V, s->Kp, s->alpha, s->beta, s->D, s->doc_off, s->z, s->nw,
                        s->nwsum, doc_part, word_part);
}

double orc_exact_log_likelihood(const orc_exact* s) {
  return mallet_ll_dense(s->K, s->V, s->Kp, s->alpha, s->beta, s->D, s->doc_off, s->z, s->nw,
                         s->nwsum);
}

void orc_exact_infer(const orc_exact* s, int64_t Dh, const int64_t* doc_off, const int32_t* words,
                     int32_t n_iter, int32_t burn_in, int32_t thin, uint64_t seed, double* theta) {
  /* TopicInferencer skips tokens whose type has no training tokens (an empty
   * typeTopicCounts row): keep only tokens of words with a nonzero total */
  const int64_t N_in = doc_off[Dh] - doc_off[0];
  int64_t* off = (int64_t*)malloc(sizeof(int64_t) * (Dh + 1));
  int32_t* w = (int32_t*)malloc(sizeof(int32_t) * (N_in ? N_in : 1));
  int64_t N = 0;
  off[0] = 0;
  for (int64_t d = 0; d < Dh; ++d) {
    for (int64_t i = doc_off[d] - doc_off[0]; i < doc_off[d + 1] - doc_off[0]; ++i) {
      const int32_t* row = s->nw + (size_t)words[i] * s->Kp;
      int64_t tot = 0;
      for (int k = 0; k < s->K; ++k) tot += row[k];
      if (tot > 0) w[N++] = words[i];
    }
    off[d + 1] = N;
  }
  int32_t* z = (int32_t*)malloc(sizeof(int32_t) * (N ? N : 1));
  /* TopicInferencer init: the most frequent topic of the word in the model
   * (packed rows are sorted by (count << bits | topic), so ties go to the
   * larger topic id). */
  for (int64_t i = 0; i < N; ++i) {
    const int32_t* row = s->nw + (size_t)w[i] * s->Kp;
    int best = 0;
    for (int k = 1; k < s->K; ++k)
      if (row[k] >= row[best]) best = k;
    z[i] = best;
  }
  int64_t* acc = (int64_t*)calloc((size_t)Dh * s->K, sizeof(int64_t));
  int32_t nsamples = 0;
  orc_exact tmp = *s;
  tmp.seed = seed;
  for (int32_t it = 1; it <= n_iter; ++it) {
    exact_sample_stream(&tmp, off, w, z, Dh, 1, (uint32_t)(it - 1), STREAM_INFER, 0, NULL);
    if (it > burn_in && (it - burn_in) % thin == 0) {
      nsamples++;
      for (int64_t d = 0; d < Dh; ++d)
        for (int64_t i = off[d]; i < off[d + 1]; ++i) acc[(size_t)d * s->K + z[i]]++;
    }
  }
  if (nsamples == 0) {
    nsamples = 1;
    for (int64_t d = 0; d < Dh; ++d)
      for (int64_t i = off[d]; i < off[d + 1]; ++i) acc[(size_t)d * s->K + z[i]]++;
  }
  for (int64_t d = 0; d < Dh; ++d) {
    double sum = 0.0;
    for (int k = 0; k < s->K; ++k) {
      double v = (double)nsamples * s->alpha[k] + (double)acc[(size_t)d * s->K + k];
      theta[(size_t)d * s->K + k] = v;
      sum += v;
    }
    for (int k = 0; k < s->K; ++k) theta[(size_t)d * s->K + k] /= sum;
  }
  free(acc);
  free(z);
  free(w);
  free(off);
}

double orc_doc_completion_loglik(int32_t K, int32_t V, const int32_t* nw, const int32_t* nwsum,
                                 double beta, int64_t Dh, const double* theta,
                                 const int64_t* doc_off, const int32_t* words) {
  double ll = 0.0;
  double vbeta = beta * V;
  for (int64_t d = 0; d < Dh; ++d) {
    const double* th = theta + (size_t)d * K;
    for (int64_t i = doc_off[d]; i < doc_off[d + 1]; ++i) {
      int w = words[i];
      double p = 0.0;
      for (int k = 0; k < K; ++k) p += th[k] * ((double)nw[(size_t)w * K + k] + beta) / ((double)nwsum[k] + vbeta);
      ll += log(p);
    }
  }
  return ll;
}

/* ======================================================================== */
/* cpu_mallet — Mallet 2.0.7 ParallelTopicModel / WorkerRunnable [M]        */
/* ======================================================================== */
typedef struct {
  int32_t** ttc;  /* typeTopicCounts[V][len[w]] packed (count<<bits)|topic */
  int32_t* tpt;   /* tokensPerTopic[K] */
  double* cached; /* cachedCoefficients[K] */
  double smoothing_only_mass;
  orc_jrandom rng;
  int64_t start_doc, num_docs;
  int32_t *local_counts, *local_index;
  double* term_scores;
  int collect;                 /* shouldSaveState: record alpha statistics */
  int32_t* doc_len_counts;     /* [max_len+1] */
  int32_t* topic_doc_counts;   /* [K][max_len+1] */
  double t_build;              /* this sweep's buildLocalTypeTopicCounts seconds */
} mallet_worker;

struct orc_mallet {
  int32_t K, V, T;
  int32_t topic_mask, topic_bits;
  double alpha_sum, beta, beta_sum;
  double* alpha;
  int64_t D, N;
  int64_t* doc_off;
  int32_t* words;
  int32_t* z;
  int32_t* type_totals;
  int32_t* row_len;
  int32_t** ttc; /* global typeTopicCounts */
  int32_t* tpt;  /* global tokensPerTopic */
  mallet_worker* workers;
  int64_t seed;
  /* hyperparameter optimisation (setOptimizeInterval / setBurninPeriod) */
  int32_t optimize_interval, burnin, save_sample_interval, symmetric_alpha;
  int32_t max_len;
  /* wall time of the sweeps' sampling (the workers' parallel section) and of
   * the sumTypeTopicCounts merge (orc_mallet_timing; bench.py cpu_baseline) */
  double t_sample, t_merge;
  double t_build;   /* per sweep, the slowest worker's buildLocalTypeTopicCounts */
  int pin_threads;   /* 1: worker t pinned to the t-th CPU of the affinity mask */
};

static int32_t** ttc_alloc(const orc_mallet* m) {
  int32_t** t = (int32_t**)malloc(sizeof(int32_t*) * m->V);
  for (int w = 0; w < m->V; ++w) t[w] = (int32_t*)calloc(m->row_len[w] ? m->row_len[w] : 1, sizeof(int32_t));
  return t;
}
static void ttc_free(const orc_mallet* m, int32_t** t) {
  for (int w = 0; w < m->V; ++w) free(t[w]);
  free(t);
}

/* buildInitialTypeTopicCounts / WorkerRunnable.buildLocalTypeTopicCounts:
 * add one (type, topic) occurrence to a packed row, keeping it sorted. */
static void ttc_add_one(const orc_mallet* m, int32_t* row, int len, int topic) {
  int index = 0;
  int current_topic = row[index] & m->topic_mask;
  while (row[index] > 0 && current_topic != topic) {
    index++;
    if (index == len) return; /* Mallet logs "overflow"; cannot happen: len >= distinct topics */
    current_topic = row[index] & m->topic_mask;
  }
  int current_value = row[index] >> m->topic_bits;
  if (current_value == 0) {
    row[index] = (1 << m->topic_bits) + topic;
  } else {
    row[index] = ((current_value + 1) << m->topic_bits) + topic;
    while (index > 0 && row[index] > row[index - 1]) {
      int32_t tmp = row[index];
      row[index] = row[index - 1];
      row[index - 1] = tmp;
      index--;
    }
  }
}

static void build_counts(const orc_mallet* m, int32_t** ttc, int32_t* tpt, int64_t d0, int64_t d1) {
  memset(tpt, 0, sizeof(int32_t) * m->K);
  for (int w = 0; w < m->V; ++w) {
    int32_t* row = ttc[w];
    for (int p = 0; p < m->row_len[w] && row[p] > 0; ++p) row[p] = 0;
  }
  for (int64_t d = d0; d < d1; ++d)
    for (int64_t i = m->doc_off[d]; i < m->doc_off[d + 1]; ++i) {
      int topic = m->z[i];
      tpt[topic]++;
      ttc_add_one(m, ttc[m->words[i]], m->row_len[m->words[i]], topic);
    }
}

orc_mallet* orc_mallet_create(int32_t K, double alpha_sum, double beta, int32_t V, int64_t D,
                              const int64_t* doc_off, const int32_t* words, int64_t seed,
                              int32_t num_threads) {
  orc_mallet* m = (orc_mallet*)calloc(1, sizeof(orc_mallet));
  m->K = K;
  m->V = V;
  m->T = num_threads < 1 ? 1 : num_threads;
  /* ParallelTopicModel(int numberOfTopics, double alphaSum, double beta) */
  if ((K & (K - 1)) == 0) {
    m->topic_mask = K - 1;
  } else {
    int hb = 1;
    while (hb * 2 <= K) hb *= 2;
    m->topic_mask = hb * 2 - 1;
  }
  m->topic_bits = __builtin_popcount((unsigned)m->topic_mask);
  m->alpha_sum = alpha_sum;
  m->beta = beta;
  m->alpha = (double*)malloc(sizeof(double) * K);
  for (int k = 0; k < K; ++k) m->alpha[k] = alpha_sum / K;
  m->D = D;
  m->N = doc_off[D] - doc_off[0];
  m->doc_off = (int64_t*)malloc(sizeof(int64_t) * (D + 1));
  for (int64_t d = 0; d <= D; ++d) m->doc_off[d] = doc_off[d] - doc_off[0];
  m->words = (int32_t*)malloc(sizeof(int32_t) * (m->N ? m->N : 1));
  memcpy(m->words, words, sizeof(int32_t) * m->N);
  m->z = (int32_t*)malloc(sizeof(int32_t) * (m->N ? m->N : 1));
  m->seed = seed;
  /* addInstances: betaSum, typeTotals, row lengths min(K, typeTotal) */
  m->beta_sum = beta * V;
  m->type_totals = (int32_t*)calloc(V, sizeof(int32_t));
  for (int64_t i = 0; i < m->N; ++i) m->type_totals[m->words[i]]++;
  m->row_len = (int32_t*)malloc(sizeof(int32_t) * V);
  for (int w = 0; w < V; ++w) m->row_len[w] = m->type_totals[w] < K ? m->type_totals[w] : K;
  m->ttc = ttc_alloc(m);
  m->tpt = (int32_t*)calloc(K, sizeof(int32_t));
  /* topics[position] = random.nextInt(numTopics), doc by doc */
  orc_jrandom r;
  orc_jrandom_seed(&r, seed);
  for (int64_t i = 0; i < m->N; ++i) m->z[i] = orc_jrandom_next_int_n(&r, K);
  build_counts(m, m->ttc, m->tpt, 0, D);
  /* estimate(): runnables with contiguous doc blocks; last takes the rest */
  m->workers = (mallet_worker*)calloc(m->T, sizeof(mallet_worker));
  int64_t per = D / m->T, offset = 0;
  for (int t = 0; t < m->T; ++t) {
    mallet_worker* wk = &m->workers[t];
    wk->start_doc = offset;
    wk->num_docs = (t == m->T - 1) ? D - offset : per;
    offset += wk->num_docs;
    if (m->T > 1) {
      wk->ttc = ttc_alloc(m);
      for (int w = 0; w < V; ++w) memcpy(wk->ttc[w], m->ttc[w], sizeof(int32_t) * m->row_len[w]);
      wk->tpt = (int32_t*)malloc(sizeof(int32_t) * K);
      memcpy(wk->tpt, m->tpt, sizeof(int32_t) * K);
    } else {
      wk->ttc = m->ttc;
      wk->tpt = m->tpt;
    }
    wk->cached = (double*)calloc(K, sizeof(double));
    wk->local_counts = (int32_t*)calloc(K, sizeof(int32_t));
    wk->local_index = (int32_t*)calloc(K, sizeof(int32_t));
    wk->term_scores = (double*)calloc(K, sizeof(double));
    orc_jrandom_seed(&wk->rng, seed);
  }
  m->burnin = 200;
  m->save_sample_interval = 10;
  m->max_len = 0;
  for (int64_t d = 0; d < D; ++d)
    if (m->doc_off[d + 1] - m->doc_off[d] > m->max_len) m->max_len = (int32_t)(m->doc_off[d + 1] - m->doc_off[d]);
  for (int t = 0; t < m->T; ++t) {
    m->workers[t].doc_len_counts = (int32_t*)calloc(m->max_len + 1, sizeof(int32_t));
    m->workers[t].topic_doc_counts = (int32_t*)calloc((size_t)K * (m->max_len + 1), sizeof(int32_t));
  }
  return m;
}

void orc_mallet_set_optimize(orc_mallet* m, int32_t interval, int32_t burnin, int32_t symmetric) {
  m->optimize_interval = interval;
  m->burnin = burnin;
  m->symmetric_alpha = symmetric;
}

void orc_mallet_get_hyper(const orc_mallet* m, double* alpha, double* beta) {
  if (alpha) memcpy(alpha, m->alpha, sizeof(double) * m->K);
  if (beta) *beta = m->beta;
}

/* ParallelTopicModel.optimizeAlpha [M] */
static void mallet_optimize_alpha(orc_mallet* m) {
  const int64_t W = (int64_t)m->max_len + 1;
  int32_t* lens = (int32_t*)calloc(W, sizeof(int32_t));
  int32_t* hist = (int32_t*)calloc((size_t)m->K * W, sizeof(int32_t));
  for (int t = 0; t < m->T; ++t) {
    mallet_worker* wk = &m->workers[t];
    for (int64_t i = 0; i < W; ++i) {
      lens[i] += wk->doc_len_counts[i];
      wk->doc_len_counts[i] = 0;
    }
    for (int k = 0; k < m->K; ++k)
      for (int64_t i = 0; i < W; ++i) {
        /* symmetric alpha pools every topic into row 0 */
        hist[(m->symmetric_alpha ? 0 : k) * W + i] += wk->topic_doc_counts[k * W + i];
        wk->topic_doc_counts[k * W + i] = 0;
      }
  }
  if (m->symmetric_alpha) {
    m->alpha_sum = orc_learn_symmetric_concentration(hist, W - 1, lens, W - 1, m->K, m->alpha_sum);
    for (int k = 0; k < m->K; ++k) m->alpha[k] = m->alpha_sum / m->K;
  } else {
    m->alpha_sum = orc_learn_parameters(m->alpha, m->K, hist, lens, m->max_len, 1.001, 1.0, 1);
  }
  free(lens);
  free(hist);
}

/* ParallelTopicModel.optimizeBeta [M] */
static void mallet_optimize_beta(orc_mallet* m) {
  int32_t max_type = 0, max_topic = 0;
  for (int w = 0; w < m->V; ++w)
    if (m->type_totals[w] > max_type) max_type = m->type_totals[w];
  for (int k = 0; k < m->K; ++k)
    if (m->tpt[k] > max_topic) max_topic = m->tpt[k];
  int32_t* counts = (int32_t*)calloc((size_t)max_type + 1, sizeof(int32_t));
  int32_t* sizes = (int32_t*)calloc((size_t)max_topic + 1, sizeof(int32_t));
  for (int w = 0; w < m->V; ++w)
    for (int p = 0; p < m->row_len[w] && m->ttc[w][p] > 0; ++p) counts[m->ttc[w][p] >> m->topic_bits]++;
  for (int k = 0; k < m->K; ++k) sizes[m->tpt[k]]++;
  m->beta_sum = orc_learn_symmetric_concentration(counts, max_type, sizes, max_topic, m->V, m->beta_sum);
  m->beta = m->beta_sum / m->V;
  free(counts);
  free(sizes);
}

void orc_mallet_destroy(orc_mallet* m) {
  if (!m) return;
  for (int t = 0; t < m->T; ++t) {
    mallet_worker* wk = &m->workers[t];
    if (m->T > 1) {
      ttc_free(m, wk->ttc);
      free(wk->tpt);
    }
    free(wk->cached); free(wk->local_counts); free(wk->local_index); free(wk->term_scores);
    free(wk->doc_len_counts); free(wk->topic_doc_counts);
  }
  free(m->workers);
  ttc_free(m, m->ttc);
  free(m->tpt); free(m->alpha); free(m->doc_off); free(m->words); free(m->z);
  free(m->type_totals); free(m->row_len);
  free(m);
}

/* WorkerRunnable.sampleTopicsForOneDoc [M] */
static void mallet_sample_doc(const orc_mallet* m, mallet_worker* wk, int64_t d) {
  const int K = m->K;
  const int32_t mask = m->topic_mask, bits = m->topic_bits;
  const double beta = m->beta, beta_sum = m->beta_sum;
  const double* alpha = m->alpha;
  int32_t* tpt = wk->tpt;
  double* cached = wk->cached;
  int32_t* lc = wk->local_counts;
  int32_t* li = wk->local_index;
  double* scores = wk->term_scores;
  int32_t* topics = m->z + m->doc_off[d];
  const int32_t* tokens = m->words + m->doc_off[d];
  int64_t len = m->doc_off[d + 1] - m->doc_off[d];

  memset(lc, 0, sizeof(int32_t) * K);
  for (int64_t p = 0; p < len; ++p) lc[topics[p]]++;
  int dense = 0;
  for (int k = 0; k < K; ++k)
    if (lc[k] != 0) li[dense++] = k;
  int nonzero = dense;
  double topic_beta_mass = 0.0;
  for (dense = 0; dense < nonzero; ++dense) {
    int k = li[dense];
    int n = lc[k];
    topic_beta_mass += beta * n / (tpt[k] + beta_sum);
    cached[k] = (alpha[k] + n) / (tpt[k] + beta_sum);
  }
  for (int64_t p = 0; p < len; ++p) {
    int type = tokens[p];
    int old_topic = topics[p];
    int32_t* row = wk->ttc[type];
    int row_len = m->row_len[type];
    /* remove this token from all counts */
    wk->smoothing_only_mass -= alpha[old_topic] * beta / (tpt[old_topic] + beta_sum);
    topic_beta_mass -= beta * lc[old_topic] / (tpt[old_topic] + beta_sum);
    lc[old_topic]--;
    if (lc[old_topic] == 0) {
      dense = 0;
      while (li[dense] != old_topic) dense++;
      while (dense < nonzero) {
        if (dense < K - 1) li[dense] = li[dense + 1];
        dense++;
      }
      nonzero--;
    }
    tpt[old_topic]--;
    wk->smoothing_only_mass += alpha[old_topic] * beta / (tpt[old_topic] + beta_sum);
    topic_beta_mass += beta * lc[old_topic] / (tpt[old_topic] + beta_sum);
    cached[old_topic] = (alpha[old_topic] + lc[old_topic]) / (tpt[old_topic] + beta_sum);

    /* walk the packed row: decrement the old topic, score the rest */
    int index = 0;
    int already_decremented = 0;
    double topic_term_mass = 0.0;
    while (index < row_len && row[index] > 0) {
      int current_topic = row[index] & mask;
      int current_value = row[index] >> bits;
      if (!already_decremented && current_topic == old_topic) {
        current_value--;
        if (current_value == 0)
          row[index] = 0;
        else
          row[index] = (current_value << bits) + old_topic;
        int sub = index;
        while (sub < row_len - 1 && row[sub] < row[sub + 1]) {
          int32_t tmp = row[sub];
          row[sub] = row[sub + 1];
          row[sub + 1] = tmp;
          sub++;
        }
        already_decremented = 1;
      } else {
        double score = cached[current_topic] * current_value;
        topic_term_mass += score;
        scores[index] = score;
        index++;
      }
    }
    double sample = orc_jrandom_next_double(&wk->rng) *
                    (wk->smoothing_only_mass + topic_beta_mass + topic_term_mass);
    int new_topic = -1;
    if (sample < topic_term_mass) {
      int i = -1;
      while (sample > 0) {
        i++;
        sample -= scores[i];
      }
      new_topic = row[i] & mask;
      int current_value = row[i] >> bits;
      row[i] = ((current_value + 1) << bits) + new_topic;
      while (i > 0 && row[i] > row[i - 1]) {
        int32_t tmp = row[i];
        row[i] = row[i - 1];
        row[i - 1] = tmp;
        i--;
      }
    } else {
      sample -= topic_term_mass;
      if (sample < topic_beta_mass) {
        sample /= beta;
        for (dense = 0; dense < nonzero; ++dense) {
          int k = li[dense];
          sample -= lc[k] / (tpt[k] + beta_sum);
          if (sample <= 0.0) {
            new_topic = k;
            break;
          }
        }
      } else {
        sample -= topic_beta_mass;
        sample /= beta;
        new_topic = 0;
        sample -= alpha[new_topic] / (tpt[new_topic] + beta_sum);
        while (sample > 0.0 && new_topic < K - 1) {
          new_topic++;
          sample -= alpha[new_topic] / (tpt[new_topic] + beta_sum);
        }
      }
      if (new_topic == -1) new_topic = K - 1; /* "sampling error" fallback */
      index = 0;
      while (row[index] > 0 && (row[index] & mask) != new_topic) {
        index++;
        if (index == row_len) break;
      }
      if (index < row_len) {
        if (row[index] == 0) {
          row[index] = (1 << bits) + new_topic;
        } else {
          int current_value = row[index] >> bits;
          row[index] = ((current_value + 1) << bits) + new_topic;
          while (index > 0 && row[index] > row[index - 1]) {
            int32_t tmp = row[index];
            row[index] = row[index - 1];
            row[index - 1] = tmp;
            index--;
          }
        }
      }
    }
    topics[p] = new_topic;
    wk->smoothing_only_mass -= alpha[new_topic] * beta / (tpt[new_topic] + beta_sum);
    topic_beta_mass -= beta * lc[new_topic] / (tpt[new_topic] + beta_sum);
    lc[new_topic]++;
    if (lc[new_topic] == 1) {
      dense = nonzero;
      while (dense > 0 && li[dense - 1] > new_topic) {
        li[dense] = li[dense - 1];
        dense--;
      }
      li[dense] = new_topic;
      nonzero++;
    }
    tpt[new_topic]++;
    cached[new_topic] = (alpha[new_topic] + lc[new_topic]) / (tpt[new_topic] + beta_sum);
    wk->smoothing_only_mass += alpha[new_topic] * beta / (tpt[new_topic] + beta_sum);
    topic_beta_mass += beta * lc[new_topic] / (tpt[new_topic] + beta_sum);
  }
  if (wk->collect) {
    const int64_t W = (int64_t)m->max_len + 1;
    wk->doc_len_counts[len]++;
    for (dense = 0; dense < nonzero; ++dense) wk->topic_doc_counts[li[dense] * W + lc[li[dense]]]++;
  }
  for (dense = 0; dense < nonzero; ++dense) {
    int k = li[dense];
    cached[k] = alpha[k] / (tpt[k] + beta_sum);
  }
}

typedef struct {
  orc_mallet* m;
  int t;
} mallet_job;

static double wall_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* WorkerRunnable.run() [M] */
static void* mallet_worker_run(void* arg) {
  mallet_job* job = (mallet_job*)arg;
  orc_mallet* m = job->m;
  mallet_worker* wk = &m->workers[job->t];
  wk->smoothing_only_mass = 0.0;
  for (int k = 0; k < m->K; ++k) {
    wk->smoothing_only_mass += m->alpha[k] * m->beta / (wk->tpt[k] + m->beta_sum);
    wk->cached[k] = m->alpha[k] / (wk->tpt[k] + m->beta_sum);
  }
  for (int64_t d = wk->start_doc; d < m->D && d < wk->start_doc + wk->num_docs; ++d)
    mallet_sample_doc(m, wk, d);
  if (m->T > 1) {
    const double tb = wall_s();
    build_counts(m, wk->ttc, wk->tpt, wk->start_doc, wk->start_doc + wk->num_docs);
    wk->t_build = wall_s() - tb;
  }
  return NULL;
}

/* ParallelTopicModel.sumTypeTopicCounts + copy-back to every runnable [M] */
static void mallet_sum_type_topic_counts(orc_mallet* m) {
  memset(m->tpt, 0, sizeof(int32_t) * m->K);
  for (int w = 0; w < m->V; ++w) {
    int32_t* row = m->ttc[w];
    for (int p = 0; p < m->row_len[w] && row[p] > 0; ++p) row[p] = 0;
  }
  for (int t = 0; t < m->T; ++t) {
    mallet_worker* wk = &m->workers[t];
    for (int k = 0; k < m->K; ++k) m->tpt[k] += wk->tpt[k];
    for (int w = 0; w < m->V; ++w) {
      int32_t* src = wk->ttc[w];
      int32_t* dst = m->ttc[w];
      int len = m->row_len[w];
      for (int si = 0; si < len && src[si] > 0; ++si) {
        int topic = src[si] & m->topic_mask;
        int count = src[si] >> m->topic_bits;
        int ti = 0;
        int current_topic = dst[ti] & m->topic_mask;
        while (dst[ti] > 0 && current_topic != topic) {
          ti++;
          current_topic = dst[ti] & m->topic_mask;
        }
        int current_count = dst[ti] >> m->topic_bits;
        dst[ti] = ((current_count + count) << m->topic_bits) + topic;
        while (ti > 0 && dst[ti] > dst[ti - 1]) {
          int32_t tmp = dst[ti];
          dst[ti] = dst[ti - 1];
          dst[ti - 1] = tmp;
          ti--;
        }
      }
    }
  }
  for (int t = 0; t < m->T; ++t) {
    mallet_worker* wk = &m->workers[t];
    memcpy(wk->tpt, m->tpt, sizeof(int32_t) * m->K);
    for (int w = 0; w < m->V; ++w) {
      int32_t* dst = wk->ttc[w];
      int32_t* src = m->ttc[w];
      for (int p = 0; p < m->row_len[w]; ++p) {
        if (src[p] != 0)
          dst[p] = src[p];
        else if (dst[p] != 0)
          dst[p] = 0;
        else
          break;
      }
    }
  }
}

void orc_mallet_set_pin_threads(orc_mallet* m, int32_t on) { m->pin_threads = on; }
void orc_mallet_timing(orc_mallet* m, double* sample_s, double* merge_s, int32_t reset) {
  if (sample_s) *sample_s = m->t_sample;
  if (merge_s) *merge_s = m->t_merge;
  if (reset) m->t_sample = m->t_merge = m->t_build = 0.0;
}
/* the part of the timed sampling phase spent in the workers'
 * buildLocalTypeTopicCounts (the slowest worker's, summed over sweeps) */
void orc_mallet_timing_build(const orc_mallet* m, double* build_s) { *build_s = m->t_build; }

void orc_mallet_estimate(orc_mallet* m, int32_t n_iter) {
  mallet_job* jobs = (mallet_job*)malloc(sizeof(mallet_job) * m->T);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * m->T);
  /* the CPUs this process may run on, for pinning worker t to the t-th */
  cpu_set_t mask;
  int ncpu = 0, cpus[1024];
  if (m->pin_threads && sched_getaffinity(0, sizeof mask, &mask) == 0)
    for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; ++c)
      if (CPU_ISSET(c, &mask)) cpus[ncpu++] = c;
  for (int it = 1; it <= n_iter; ++it) {
    const int opt_on = it > m->burnin && m->optimize_interval != 0;
    for (int t = 0; t < m->T; ++t) m->workers[t].collect = opt_on && it % m->save_sample_interval == 0;
    const double t0 = wall_s();
    if (m->T > 1) {
      for (int t = 0; t < m->T; ++t) {
        jobs[t].m = m;
        jobs[t].t = t;
        pthread_attr_t at;
        pthread_attr_init(&at);
        if (ncpu > 0) {
          cpu_set_t one;
          CPU_ZERO(&one);
          CPU_SET(cpus[t % ncpu], &one);
          pthread_attr_setaffinity_np(&at, sizeof one, &one);
        }
        pthread_create(&th[t], &at, mallet_worker_run, &jobs[t]);
        pthread_attr_destroy(&at);
      }
      for (int t = 0; t < m->T; ++t) pthread_join(th[t], NULL);
      const double t1 = wall_s();
      double tb = 0.0;
      for (int t = 0; t < m->T; ++t) tb = m->workers[t].t_build > tb ? m->workers[t].t_build : tb;
      m->t_build += tb;
      mallet_sum_type_topic_counts(m);
      m->t_sample += t1 - t0;
      m->t_merge += wall_s() - t1;
    } else {
      jobs[0].m = m;
      jobs[0].t = 0;
      mallet_worker_run(&jobs[0]);
      m->t_sample += wall_s() - t0;
    }
    for (int t = 0; t < m->T; ++t) m->workers[t].collect = 0;
    if (opt_on && it % m->optimize_interval == 0) {
      mallet_optimize_alpha(m);
      mallet_optimize_beta(m);
    }
  }
  free(jobs);
  free(th);
}

static void mallet_dense_counts(const orc_mallet* m, int32_t* nw, int32_t* nwsum) {
  if (nw) {
    memset(nw, 0, sizeof(int32_t) * (size_t)m->V * m->K);
    for (int w = 0; w < m->V; ++w)
      for (int p = 0; p < m->row_len[w] && m->ttc[w][p] > 0; ++p)
        nw[(size_t)w * m->K + (m->ttc[w][p] & m->topic_mask)] = m->ttc[w][p] >> m->topic_bits;
  }
  if (nwsum) memcpy(nwsum, m->tpt, sizeof(int32_t) * m->K);
}

double orc_mallet_log_likelihood(const orc_mallet* m) {
  int32_t* nw = (int32_t*)malloc(sizeof(int32_t) * (size_t)m->V * m->K);
  mallet_dense_counts(m, nw, NULL);
  double ll = mallet_ll_dense(m->K, m->V, m->K, m->alpha, m->beta, m->D, m->doc_off, m->z, nw, m->tpt);
  free(nw);
  return ll;
}

void orc_mallet_get_z(const orc_mallet* m, int32_t* z) { memcpy(z, m->z, sizeof(int32_t) * m->N); }

void orc_mallet_get_counts(const orc_mallet* m, int32_t* nw, int32_t* nwsum) {
  mallet_dense_counts(m, nw, nwsum);
}

/* TopicInferencer.getSampledDistribution [M] (sparse, fp64, frozen counts). */
void orc_mallet_infer(const orc_mallet* m, int64_t Dh, const int64_t* doc_off, const int32_t* words,
                      int32_t n_iter, int32_t burn_in, int32_t thin, int64_t seed, double* theta) {
  const int K = m->K;
  const int32_t mask = m->topic_mask;
  const double beta = m->beta, beta_sum = m->beta_sum;
  const double* alpha = m->alpha;
  const int32_t* tpt = m->tpt;
  int32_t** ttc = m->ttc;
  double* cached = (double*)malloc(sizeof(double) * K);
  double* scores = (double*)malloc(sizeof(double) * K);
  int32_t* lc = (int32_t*)malloc(sizeof(int32_t) * K);
  int32_t* li = (int32_t*)malloc(sizeof(int32_t) * K);
  double smoothing_only_mass = 0.0;
  for (int k = 0; k < K; ++k) {
    smoothing_only_mass += alpha[k] * beta / (tpt[k] + beta_sum);
    cached[k] = alpha[k] / (tpt[k] + beta_sum);
  }
  orc_jrandom rng;
  orc_jrandom_seed(&rng, seed);
  for (int64_t d = 0; d < Dh; ++d) {
    const int32_t* tokens = words + (doc_off[d] - doc_off[0]);
    int64_t len = doc_off[d + 1] - doc_off[d];
    int32_t* topics = (int32_t*)calloc(len ? len : 1, sizeof(int32_t));
    memset(lc, 0, sizeof(int32_t) * K);
    for (int64_t p = 0; p < len; ++p) {
      int type = tokens[p];
      if (type < m->V && m->row_len[type] != 0) {
        topics[p] = ttc[type][0] & mask;
        lc[topics[p]]++;
      }
    }
    int dense = 0;
    for (int k = 0; k < K; ++k)
      if (lc[k] != 0) li[dense++] = k;
    int nonzero = dense;
    double topic_beta_mass = 0.0;
    for (dense = 0; dense < nonzero; ++dense) {
      int k = li[dense];
      topic_beta_mass += beta * lc[k] / (tpt[k] + beta_sum);
      cached[k] = (alpha[k] + lc[k]) / (tpt[k] + beta_sum);
    }
    double* result = theta + (size_t)d * K;
    for (int k = 0; k < K; ++k) result[k] = 0.0;
    double sum = 0.0;
    for (int it = 1; it <= n_iter; ++it) {
      for (int64_t p = 0; p < len; ++p) {
        int type = tokens[p];
        if (type >= m->V || m->row_len[type] == 0) continue;
        int old_topic = topics[p];
        const int32_t* row = ttc[type];
        int row_len = m->row_len[type];
        topic_beta_mass -= beta * lc[old_topic] / (tpt[old_topic] + beta_sum);
        lc[old_topic]--;
        if (lc[old_topic] == 0) {
          dense = 0;
          while (li[dense] != old_topic) dense++;
          while (dense < nonzero) {
            if (dense < K - 1) li[dense] = li[dense + 1];
            dense++;
          }
          nonzero--;
        }
        topic_beta_mass += beta * lc[old_topic] / (tpt[old_topic] + beta_sum);
        cached[old_topic] = (alpha[old_topic] + lc[old_topic]) / (tpt[old_topic] + beta_sum);
        int index = 0;
        double topic_term_mass = 0.0;
        while (index < row_len && row[index] > 0) {
          int current_topic = row[index] & mask;
          int current_value = row[index] >> m->topic_bits;
          double score = cached[current_topic] * current_value;
          topic_term_mass += score;
          scores[index] = score;
          index++;
        }
        double sample = orc_jrandom_next_double(&rng) * (smoothing_only_mass + topic_beta_mass + topic_term_mass);
        int new_topic = -1;
        if (sample < topic_term_mass) {
          int i = -1;
          while (sample > 0) {
            i++;
            sample -= scores[i];
          }
          new_topic = row[i] & mask;
        } else {
          sample -= topic_term_mass;
          if (sample < topic_beta_mass) {
            sample /= beta;
            for (dense = 0; dense < nonzero; ++dense) {
              int k = li[dense];
              sample -= lc[k] / (tpt[k] + beta_sum);
              if (sample <= 0.0) {
                new_topic = k;
                break;
              }
            }
          } else {
            sample -= topic_beta_mass;
            sample /= beta;
            new_topic = 0;
            sample -= alpha[new_topic] / (tpt[new_topic] + beta_sum);
            while (sample > 0.0 && new_topic < K - 1) {
              new_topic++;
              sample -= alpha[new_topic] / (tpt[new_topic] + beta_sum);
            }
          }
        }
        if (new_topic == -1) new_topic = K - 1;
        topics[p] = new_topic;
        topic_beta_mass -= beta * lc[new_topic] / (tpt[new_topic] + beta_sum);
        lc[new_topic]++;
        if (lc[new_topic] == 1) {
          dense = nonzero;
          while (dense > 0 && li[dense - 1] > new_topic) {
            li[dense] = li[dense - 1];
            dense--;
          }
          li[dense] = new_topic;
          nonzero++;
        }
        cached[new_topic] = (alpha[new_topic] + lc[new_topic]) / (tpt[new_topic] + beta_sum);
        topic_beta_mass += beta * lc[new_topic] / (tpt[new_topic] + beta_sum);
      }
      if (it > burn_in && (it - burn_in) % thin == 0) {
        for (int k = 0; k < K; ++k) {
          result[k] += alpha[k] + lc[k];
          sum += alpha[k] + lc[k];
        }
      }
    }
    for (dense = 0; dense < nonzero; ++dense) {
      int k = li[dense];
      cached[k] = alpha[k] / (tpt[k] + beta_sum);
    }
    if (sum == 0.0) {
      for (int k = 0; k < K; ++k) {
        result[k] = alpha[k] + lc[k];
        sum += result[k];
      }
    }
    for (int k = 0; k < K; ++k) result[k] /= sum;
    free(topics);
  }
  free(cached); free(scores); free(lc); free(li);
}
