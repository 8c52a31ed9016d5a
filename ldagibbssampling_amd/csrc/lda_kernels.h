// lda_kernels.h — internal interface between the C-ABI runtime
// (lda_capi.cpp) and the gfx950 kernels (lda_kernels.hip).  Not installed.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace lda {

// Philox counter word 3: which stream a draw belongs to.
constexpr uint32_t STREAM_SAMPLE = 0u;
constexpr uint32_t STREAM_INIT = 1u;
constexpr uint32_t STREAM_INFER = 2u;

// Row-prefetch depth of the sampler per C = Kp/64 (tokens in flight per wave;
// C = 8: P = 3 is +1% over 2 on C4 once the pipeline waits vmcnt(P-1), P = 4
// spills; C = 16: 3 is within noise of 2).
#ifndef SAMPLE_P1
#define SAMPLE_P1 4
#endif
#ifndef SAMPLE_P2
#define SAMPLE_P2 4
#endif
#ifndef SAMPLE_P4
#define SAMPLE_P4 4
#endif
#ifndef SAMPLE_P8
#define SAMPLE_P8 3
#endif
#ifndef SAMPLE_P16
#define SAMPLE_P16 2
#endif
// half-wave dense sampler (K <= 128, two documents per wave): tokens in flight
#ifndef SAMPLE_PH
#define SAMPLE_PH 4
#endif
#ifndef SAMPLE_PQ
#define SAMPLE_PQ 4
#endif
// sparse sampler: tokens in flight, 64-entry rounds prefetched per token
#ifndef SPARSE_P
#define SPARSE_P 4
#endif
#ifndef SPARSE_R0
#define SPARSE_R0 2
#endif

// Per-sweep tables of the large-K sampler (k_big_tables, oracle
// exact_big_tables): the fixed-point exponent S, sum_k G_k, beta 2^-S, 2^S / beta.
struct BigScal {
  int32_t S;
  float bsig;               // beta 2^-S
  uint64_t S0;
  float bsig_hi;            // beta 2^(32-S)
  int32_t pad;
  double isig;              // 2^S / beta
};
struct BigTables {
  float2* tab;              // [Kp] {inv, ainv = alpha * inv}
  float4* tab_m1;           // [Kp] {inv_m1, alpha * inv_m1, bits of big_fix(inv_m1), bits of
                            //  big_fix(alpha inv_m1) - big_fix(alpha inv)} (0 for a topic with no tokens)
  uint32_t* F;              // [Kp] big_fix(inv)
  uint64_t* pfx;            // [Kp] inclusive prefix of big_fix(ainv)
  BigScal* scal;
};

struct SampleParams {
  const int32_t* words;     // [N] token stream (doc-contiguous)
  int32_t* z;               // [N] topic of each token (read old, write new)
  const int64_t* doc_off;   // [D+1]
  const int64_t* range_doc; // [R] work range r starts at document range_doc[r]
  const int64_t* range_end; // [R] ... and ends before range_end[r] (range_doc + 1: contiguous ranges)
  int64_t num_ranges;
  int32_t* queue;           // range counter, zeroed before each launch
  const int32_t* nw;        // [V*Kp] snapshot
  int32_t* delta;           // [V*Kp] pending nw delta
  int32_t* dsum;            // [Kp]   pending nwsum delta
  const float* alpha;       // [Kp]
  const float* inv;         // [Kp]   1/(nwsum + V*beta)
  const float* inv_m1;      // [Kp]   1/(nwsum - 1 + V*beta)
  float beta;
  int32_t K;
  int64_t token_base;       // Philox counter offset (global token index)
  uint32_t k0, k1;          // Philox key (seed)
  uint32_t c2, c3;          // Philox counter words 2 (sweep) and 3 (stream)
  // sparse rows of the snapshot (k_sample_sparse only)
  const uint32_t* ent;      // packed (count << 12) | topic, count saturated at 0xFFFFF
  const int64_t* row_off;   // [V+1] capacity offsets (min(Kp, word total) per row)
  const int32_t* row_nnz;   // [V] live entries per row; sign bit: the row has a saturated count
  const uint32_t* row_rnd;  // [V] row_off / 64 (rows start on whole 64-entry rounds)
  float* trace;             // debug only: 8 floats per token when non-null
  // 16-bit copy of the snapshot rows (k_sample)
  const uint16_t* nw16;     // [V*Kp] counts, clamped at 65535
  const uint8_t* wide;      // [V] 1 when the row holds a count > 65535 (read nw)
  // graph-launched sweeps (lda_sweep), dense kernels: [0] the sweep counter
  // (Philox word 2), which each sweep's apply advances, [1] beta's fp32 bits,
  // read from device memory in place of c2 / beta
  const uint32_t* state_dev;
  // recount sweeps of the quarter-wave sampler: the word-ordered copy of z
  // (zw[zpos[i]] = z[i], the recount index's order) kept current by the
  // sampler, so the recount streams it instead of gathering z through perm
  int32_t* zw;
  const uint32_t* zpos;
  // the large-K sampler's per-sweep tables (k_sample_big)
  BigTables big;
};

// Tokens [tok[i], tok[i+1]) of a shard belong to exchange part i.
struct PartSpans {
  int64_t tok[5];
  int32_t parts;
};
// Recount work item size: a word with more tokens in a part is split over
// several items (its row then takes device atomics).
constexpr int32_t RECOUNT_ITEM_TOKENS = 1024;

// Sparse-row packing: 12 topic bits (K <= 4096), 20 count bits; a saturated
// count field means "read the exact count from the dense nw row".
constexpr uint32_t ENT_TOPIC_BITS = 12;
constexpr uint32_t ENT_TOPIC_MASK = (1u << ENT_TOPIC_BITS) - 1;
constexpr uint32_t ENT_COUNT_SAT = (1u << (32 - ENT_TOPIC_BITS)) - 1;

// half: 1 = the half-wave variant k_sample_half, 2 = the quarter-wave
// k_sample_quarter (C <= 2 only; lda_capi.cpp: LDA_DENSE_HALF), 0 = k_sample<C>
hipError_t launch_sample(int C, bool frozen, const SampleParams& p, int blocks, hipStream_t st,
                         int half = 0);
int sample_blocks_per_cu(int C, bool frozen, int K, int half = 0);
int half_topics_per_lane(int K);
int quarter_topics_per_lane(int K);
// rb: the large-K sampler's ring (C >= 32): 0 the default depth, nonzero
// the short one for short rows (SB_RB_SHORT in lda_kernels.hip)
hipError_t launch_sample_sparse(int C, bool frozen, const SampleParams& p, int blocks,
                                hipStream_t st, int rb = 0);
constexpr int SB_RB_SHORT_ROUNDS = 6;   // the short ring's rounds (SB_RB_SHORT's default)
int sample_sparse_blocks_per_cu(int C, bool frozen);
// row totals of nw (saturating at Kp) -> host prefix -> capacity offsets
hipError_t launch_row_caps(const int32_t* nw, int64_t V, int32_t Kp, int32_t* caps, hipStream_t st);
hipError_t launch_build_sparse(const int32_t* nw, int64_t V, int32_t Kp, const int64_t* row_off,
                               uint32_t* ent, int32_t* row_nnz, hipStream_t st);
// the sparse samplers' apply + row build in one pass (rows already sized:
// build_row_capacity): nw += delta, delta = 0, dsum += the delta's column
// sums, the sparse entries and row_nnz of every row
hipError_t launch_apply_build(int32_t* nw, int32_t* delta, int64_t V, int32_t Kp, const int64_t* row_off,
                              uint32_t* ent, int32_t* row_nnz, int32_t* dsum, hipStream_t st);
// the large-K sampler's tables from the topic tables (after every k_prepare_topics)
hipError_t launch_big_tables(const int32_t* nwsum, const float* alpha_f, const float* inv, const float* inv_m1,
                             int32_t K, int32_t Kp, float beta, const BigTables& t, hipStream_t st);
hipError_t launch_build_packed(const int32_t* nw, int64_t V, int32_t Kp, uint16_t* nw16,
                               uint8_t* wide, hipStream_t st);
// per-topic state refreshed by an apply (k_prepare_topics' arguments)
struct TopicTables {
  int32_t* nwsum;           // [Kp]
  const double* alpha;      // [K]
  float* alpha_f;           // [Kp]
  float* inv;               // [Kp]
  float* inv_m1;            // [Kp]
  float vbeta;              // (float)(V * beta)
  int32_t K;
  int32_t* queue;           // work-queue counter zeroed for the next sample (nullable)
  int32_t absolute;         // 1: the buffer holds recounted counts that replace nw / nwsum
  uint32_t* state_dev;      // graph-launched sweeps: [0] advanced by one, [2] vbeta's fp32 bits read in place of vbeta
  int32_t advance;          // with state_dev: 1 = this apply ends a sweep (advance [0]); 0 = a part's apply inside one
};
// dense sampler's apply: nw += delta, delta = 0, 16-bit rows + wide flags,
// nwsum/tables (k_apply + k_build_packed + k_prepare_topics in one launch)
hipError_t launch_apply_packed(int32_t* nw, int32_t* delta, int64_t V, int32_t Kp, uint16_t* nw16,
                               uint8_t* wide, const TopicTables& t, hipStream_t st);
// the recount (see k_recount): index build and the per-sweep recount
hipError_t launch_word_hist(const int32_t* words, int64_t n, const PartSpans& ps, int64_t V,
                            uint32_t* cnt, hipStream_t st);
hipError_t launch_word_scatter(const int32_t* words, int64_t n, const PartSpans& ps, int64_t V,
                               uint32_t* cursor, uint32_t* perm, hipStream_t st);
// zpos[perm[j]] = j; zw[j] = z[perm[j]] (the word-ordered copy of z)
hipError_t launch_zw_build(const uint32_t* perm, int64_t n, const int32_t* z, uint32_t* zpos, int32_t* zw,
                           hipStream_t st);
// zw non-null: the topics are read from zw[perm index] (streamed) instead of z[perm[.]]
hipError_t launch_recount(int32_t Kp, const uint32_t* perm, const int32_t* zw, const int32_t* items, int32_t n_items,
                          const int32_t* z, int32_t* buf, int32_t* bufsum, int blocks, hipStream_t st);
hipError_t launch_philox_draws(const int64_t* gtok, int64_t n, uint32_t c2, uint32_t c3, uint64_t seed,
                               uint32_t* out, hipStream_t st);
hipError_t launch_init_z(int32_t* z, int64_t n, int32_t K, int64_t token_base, uint32_t k0,
                         uint32_t k1, hipStream_t st);
#ifdef SB_X_DELTA_KERNEL
hipError_t launch_delta_from_z(const int32_t* words, const int32_t* zold, const int32_t* z, int64_t n,
                               int32_t Kp, int32_t* delta, hipStream_t st);
#endif
hipError_t launch_count(const int32_t* words, const int32_t* z, int64_t n, int32_t Kp,
                        int32_t* delta, int32_t* dsum, hipStream_t st);
hipError_t launch_apply(int32_t* nw, int32_t* delta, int64_t n, hipStream_t st);
// dst += src; src = 0 over n int32 (n a multiple of 4): a split sweep's parts
// sparse samplers' apply: nw += delta, delta = 0, dsum += the delta's column
// sums (dsum must hold only what is to be added: the caller zeroes it)
hipError_t launch_apply_cols(int32_t* nw, int32_t* delta, int64_t V, int32_t Kp, int32_t* dsum,
                             hipStream_t st);
// compact exchange (lda_exchange_pack / _unpack): 2 cells per int32 word,
// biases b0 = 2^15 / world (bits 0..15) and b1 = 2^14 / world (bits 16..30)
inline int32_t exch_bias0(int32_t world) { return 32768 / world; }
inline int32_t exch_bias1(int32_t world) { return 16384 / world; }
// ... or 4 cells per word (lda_set_exchange_cells 4, round 6): cells 4i..4i+2
// biased by 2^7 / world in bits 0..7, 8..15, 16..23, cell 4i+3 by 2^6 / world
// in bits 24..30 (world <= 64)
inline int32_t exch_bias4(int32_t world) { return 128 / world; }
inline int32_t exch_bias4_top(int32_t world) { return 64 / world; }
// cells: a multiple of 4; packed: cells / per_word words; esc: [1 + 3 cap] with esc[0] zeroed
hipError_t launch_exch_pack(const int32_t* buf, int64_t cells, int32_t* packed, int32_t world,
                            int32_t* esc, int32_t cap, hipStream_t st, int32_t per_word = 2);
// buf[cells] = the unpacked sum, then + every rank's escapes (esc_all: world x
// [1 + 3 cap]; nullptr: none)
hipError_t launch_exch_unpack(const int32_t* packed, int64_t cells, int32_t* buf, int32_t world,
                              const int32_t* esc_all, int32_t cap, hipStream_t st, int32_t per_word = 2);
// one uint64 partial per block of the nw / nwsum hash (lda_counts_checksum)
hipError_t launch_counts_checksum(const int32_t* nw, const int32_t* nwsum, int32_t K, int32_t Kp, int64_t V,
                                  uint64_t* partial, int blocks, hipStream_t st);
hipError_t launch_fold_delta(int32_t* dst, int32_t* src, int64_t n, hipStream_t st);
hipError_t launch_prepare_topics(int32_t* nwsum, int32_t* dsum, const double* alpha, double beta,
                                 double vbeta, int32_t K, int32_t Kp, float* alpha_f, float* inv,
                                 float* inv_m1, hipStream_t st);
hipError_t launch_doc_topics(const int32_t* z, const int64_t* doc_off, int64_t D, int32_t K,
                             int32_t Kp, int32_t* out, int accumulate, hipStream_t st);
hipError_t launch_ll_docs(const int32_t* z, const int64_t* doc_off, int64_t D, const double* alpha,
                          double alpha_sum, int32_t K, int32_t Kp, double* partial, int blocks,
                          hipStream_t st);
hipError_t launch_ll_words(const int32_t* nw, int64_t V, int32_t K, int32_t Kp, double beta,
                           double* partial, unsigned long long* nonzero, int blocks,
                           hipStream_t st);
// range workers per block of the sampler kernel used for (C, sampler): 4
// waves, 16 for the large-K sparse kernel (C >= 32), 8 for the half-wave
// dense kernel (4 waves x 2 halves)
int sample_waves_per_block(int C, bool sparse, int half = 0);
hipError_t launch_row_stats(const int32_t* nw, int64_t V, int32_t K, int32_t Kp,
                            unsigned long long* out, hipStream_t st);
hipError_t launch_doc_hist(const int32_t* z, const int64_t* doc_off, int64_t D, int32_t K, int32_t Kp,
                           int32_t L, int32_t* len_hist, int32_t* topic_hist, hipStream_t st);
hipError_t launch_count_hist(const int32_t* nw, int64_t V, int32_t K, int32_t Kp, int64_t max_count,
                             int32_t* hist, int32_t* overflow, hipStream_t st);
hipError_t launch_infer_init(const int32_t* words, int32_t* z, int64_t n, const int32_t* nw,
                             int32_t K, int32_t Kp, hipStream_t st);

}  // namespace lda
