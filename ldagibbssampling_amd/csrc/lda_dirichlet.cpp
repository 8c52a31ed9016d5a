// lda_dirichlet.cpp — host-side hyperparameter estimation.
//
// The reference enables Mallet's optimisation in both drivers
// (setOptimizeInterval(20): src/cmu_ron/TrainAndPredict.java:163,
// src/cmu/TrainAndPredict.java:261).  Mallet 2.0.7 (cc.mallet:mallet:2.0.7,
// pom.xml:107-111, not vendored) runs, every optimizeInterval sweeps after the
// burn-in:
//   optimizeAlpha -> Dirichlet.learnParameters(alpha, topicDocCounts,
//                    docLengthCounts, shape 1.001, scale 1.0, 1 iteration)
//   optimizeBeta  -> Dirichlet.learnSymmetricConcentration(countHistogram,
//                    topicSizeHistogram, numTypes, betaSum), beta = betaSum/V
// Both are Minka's fixed-point updates for Dirichlet-multinomial parameters
// (T. Minka, "Estimating a Dirichlet distribution", 2000), evaluated on
// integer histograms.  The histograms come from the GPU (lda_doc_topic_histograms,
// lda_count_histogram); this file is the fp64 arithmetic, restated from the
// published algorithm.  Its independent restatement for the tests lives in
// oracle/lda_oracle.c (orc_learn_parameters, orc_learn_symmetric_concentration).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/lda_mi355x.h"
#include "lda_guard.h"

namespace {

// Dirichlet.digamma: shift the argument above 9.5, then the asymptotic series
// log z - 1/(2z) - sum_j B_2j / (2j z^2j); tiny arguments use
// psi(z) ~ -gamma - 1/z.
double digamma(double z) {
  constexpr double kEulerMascheroni = -0.5772156649015328606065121;  // -gamma
  constexpr double kSmall = 1e-6, kLarge = 9.5;
  constexpr double c1 = 1.0 / 12, c2 = 1.0 / 120, c3 = 1.0 / 252, c4 = 1.0 / 240,
                   c5 = 1.0 / 132, c6 = 691.0 / 32760, c7 = 1.0 / 12;
  if (z < kSmall) return kEulerMascheroni - 1.0 / z;
  double psi = 0.0;
  while (z < kLarge) {
    psi -= 1.0 / z;
    z += 1.0;
  }
  const double iz = 1.0 / z, iz2 = iz * iz;
  psi += std::log(z) - 0.5 * iz -
         iz2 * (c1 - iz2 * (c2 - iz2 * (c3 - iz2 * (c4 - iz2 * (c5 - iz2 * (c6 - iz2 * c7))))));
  return psi;
}

// Two deliberate departures from Mallet's literal arithmetic (both no-ops for
// ordinary values): the digamma steps add the integer offset first,
// 1/(a + (i-1)), because Java's (a + i) - 1 cancels to 0 once a < 1.1e-16 --
// which happens to topics that die under optimisation (K = 500, alphaSum =
// 100 on a small corpus) -- and turns alpha into inf/NaN; and an updated
// alpha_k is floored at 1e-300 so that a dead topic cannot underflow to 0
// over thousands of sweeps (0 * inf again).
constexpr double kMinParameter = 1e-300;

}  // namespace

extern "C" {

double lda_digamma(double z) { return digamma(z); }

lda_status lda_learn_parameters(double* params, int32_t K, const int32_t* observations,
                                const int32_t* observation_lengths, int32_t max_len, double shape,
                                double scale, int32_t iterations, double* params_sum) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!params || !observations || !observation_lengths || K < 1 || max_len < 0 || iterations < 0)
    return LDA_ERR_INVALID_ARG;
  const int64_t L1 = (int64_t)max_len + 1;
  double psum = 0.0;
  for (int k = 0; k < K; ++k) psum += params[k];
  // last index with a non-zero count in each topic's histogram (-1: none)
  std::vector<int64_t> last = lda_abi::host_vector<int64_t>((size_t)K, -1);
  for (int k = 0; k < K; ++k)
    for (int64_t i = 0; i < L1; ++i)
      if (observations[k * L1 + i] > 0) last[k] = i;
  for (int it = 0; it < iterations; ++it) {
    // denominator: sum over document lengths n of count(n) * (psi(S+n) - psi(S)),
    // the digamma difference accumulated term by term, minus 1/scale
    double denom = 0.0, dig = 0.0;
    for (int64_t n = 1; n < L1; ++n) {
      dig += 1.0 / (psum + (double)(n - 1));
      denom += (double)observation_lengths[n] * dig;
    }
    denom -= 1.0 / scale;
    psum = 0.0;
    for (int k = 0; k < K; ++k) {
      const double old = params[k];
      double num = 0.0;
      dig = 0.0;
      for (int64_t i = 1; i <= last[k]; ++i) {
        dig += 1.0 / (old + (double)(i - 1));
        num += (double)observations[k * L1 + i] * dig;
      }
      params[k] = std::max(old * (num + shape) / denom, kMinParameter);
      psum += params[k];
    }
  }
  if (params_sum) *params_sum = psum;
  return psum < 0.0 ? LDA_ERR_INVALID_ARG : LDA_OK;
  });
}

lda_status lda_learn_symmetric_concentration(const int32_t* count_hist, int64_t max_count,
                                             const int64_t* lengths, const int32_t* length_counts,
                                             int64_t n_lengths, int32_t num_dims, double current,
                                             double* out) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!count_hist || !out || max_count < 0 || n_lengths < 0 || num_dims < 1 ||
      (n_lengths > 0 && (!lengths || !length_counts)))
    return LDA_ERR_INVALID_ARG;
  int64_t top = 0;  // largest count with a non-zero histogram entry
  for (int64_t c = 0; c <= max_count; ++c)
    if (count_hist[c] > 0) top = c;
  // only non-zero observation lengths, ascending
  std::vector<int64_t> len;
  std::vector<int32_t> cnt;
  for (int64_t j = 0; j < n_lengths; ++j) {
    if (j > 0 && lengths[j] <= lengths[j - 1]) return LDA_ERR_INVALID_ARG;
    if (length_counts[j] > 0) {
      len.push_back(lengths[j]);
      cnt.push_back(length_counts[j]);
    }
  }
  // non-zero counts, ascending: the numerator walks them the way Mallet's
  // denominator walks the observation lengths (term by term across short
  // gaps, a digamma difference across gaps > 20), so its cost is the number
  // of distinct counts, not the largest count (C4: cells of ~1e5-1e6)
  std::vector<int64_t> cidx;
  for (int64_t c = 1; c <= top; ++c)
    if (count_hist[c] > 0) cidx.push_back(c);
  double value = current;
  for (int it = 1; it <= 200; ++it) {
    const double per_dim = value / num_dims;
    double dig = 0.0, num = 0.0;
    {
      const double pbase = digamma(per_dim);
      int64_t prev = 0;
      for (int64_t c : cidx) {
        if (c - prev > 20) {
          dig = digamma(per_dim + (double)c) - pbase;
        } else {
          for (int64_t i = prev + 1; i <= c; ++i) dig += 1.0 / (per_dim + (double)(i - 1));
        }
        num += (double)count_hist[c] * dig;
        prev = c;
      }
    }
    // sum over lengths n of count(n) * (psi(value + n) - psi(value)); far
    // jumps (> 20) restart from digamma differences, near ones step term by term
    dig = 0.0;
    double denom = 0.0;
    int64_t prev = 0;
    const double base = digamma(value);
    for (size_t j = 0; j < len.size(); ++j) {
      const int64_t n = len[j];
      if (n - prev > 20) {
        dig = digamma(value + (double)n) - base;
      } else {
        for (int64_t i = prev; i < n; ++i) dig += 1.0 / (value + (double)i);
      }
      denom += dig * (double)cnt[j];
      prev = n;
    }
    value = per_dim * num / denom;
  }
  *out = value;
  return LDA_OK;
  });
}

}  // extern "C"
