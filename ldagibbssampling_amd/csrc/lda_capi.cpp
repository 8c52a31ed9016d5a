// lda_capi.cpp — the C ABI (include/lda_mi355x.h) over the gfx950 kernels.
//
// One lda_ctx = one document shard on one GPU.  Device layout:
//   words[N] int32, z[N] int32           token stream, documents contiguous
//   doc_off[D+1] int64, range_doc[R+1]   documents / work ranges
//   nw[V*Kp] int32 (row = word type, Kp = K rounded up to 64), nwsum[Kp]
//   delta[V*Kp + Kp] int32               pending nw / nwsum changes (the
//                                        buffer an AD-LDA all-reduce sums)
//   alpha_f/inv/inv_m1[Kp] fp32          per-topic tables of the snapshot
// Mallet equivalents: nw ~ typeTopicCounts, nwsum ~ tokensPerTopic, z ~
// TopicAssignment.topicSequence, nd ~ WorkerRunnable.localTopicCounts (never
// stored: rebuilt from z per document inside the kernel).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <cstdlib>
#include <vector>

#include "../../include/lda_mi355x.h"
#include "lda_guard.h"
#include "lda_kernels.h"

namespace {

thread_local std::string g_last_error;
thread_local int32_t g_fail_alloc = 0;   // lda_debug_fail_host_alloc countdown (0 = off)

lda_status fail(lda_status code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define HIP_TRY(expr)                                                                     \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(e_ == hipErrorOutOfMemory ? LDA_ERR_OUT_OF_MEMORY : LDA_ERR_DEVICE,     \
                  std::string(#expr) + ": " + hipGetErrorString(e_));                     \
  } while (0)

// Kp = 64 * C with C a power of two (1..64): one kernel instantiation per C.
int pad_topics(int K) {
  int kp = 64;
  while (kp < K) kp *= 2;
  return kp;
}

double log_gamma_stirling(double z) {  // Dirichlet.logGammaStirling [M]
  const double HALF_LOG_TWO_PI = 0.91893853320467274178;
  int shift = 0;
  while (z < 2) {
    z += 1.0;
    ++shift;
  }
  double result = HALF_LOG_TWO_PI + (z - 0.5) * std::log(z) - z + 1 / (12 * z) -
                  1 / (360 * z * z * z) + 1 / (1260 * z * z * z * z * z);
  while (shift > 0) {
    --shift;
    z -= 1.0;
    result -= std::log(z);
  }
  return result;
}

// Group whole documents into work ranges of about `target` tokens.  The
// queue hands ranges out in order, so the last ~1/8 of the tokens go in
// ranges of target/4: the waves that take them finish closer together
// (a shorter launch tail).
std::vector<int64_t> make_ranges(const std::vector<int64_t>& off, int64_t target) {
  std::vector<int64_t> r;
  const int64_t D = (int64_t)off.size() - 1;
  r.push_back(0);
  int64_t start_tok = off[0];
  const int64_t tail_from = off[0] + (off[D] - off[0]) / 8 * 7;
  const int64_t tail_target = std::max<int64_t>(16, target / 4);
  for (int64_t d = 0; d < D; ++d) {
    const int64_t tgt = start_tok >= tail_from ? tail_target : target;
    if (off[d + 1] - start_tok >= tgt) {
      r.push_back(d + 1);
      start_tok = off[d + 1];
    }
  }
  if (r.back() != D) r.push_back(D);
  return r;
}

// Document cuts of `parts` token-balanced parts of a corpus whose tokens are
// global indices [g0, g0 + gn), seen from a shard whose documents start at
// global token base + off[d]: cut i (0 < i < parts) is the first local
// document starting at or after g0 + gn * i / parts.  With (g0, gn) = the
// shard itself these are the shard's own cuts; with the whole corpus every
// shard cuts where a single context over all of it would.
std::vector<int64_t> part_cuts(const std::vector<int64_t>& off, int parts, int64_t base, int64_t g0,
                               int64_t gn) {
  const int64_t D = (int64_t)off.size() - 1;
  std::vector<int64_t> cuts{0};
  for (int i = 1; i < parts; ++i) {
    const int64_t tgt = g0 + gn * i / parts - base;
    int64_t d = std::lower_bound(off.begin(), off.end(), tgt) - off.begin();
    cuts.push_back(std::min(std::max(d, cuts.back()), D));
  }
  cuts.push_back(D);
  return cuts;
}

// The work ranges of documents cut into parts (cuts[0] = 0 .. cuts[P] = D),
// each part grouped by make_ranges on its own (its own short tail).
// part_range[i] is the index of part i's first range.
std::vector<int64_t> make_cut_ranges(const std::vector<int64_t>& off, int64_t target,
                                     const std::vector<int64_t>& cuts, std::vector<int64_t>& part_range) {
  std::vector<int64_t> r{0};
  part_range.assign(1, 0);
  for (size_t i = 0; i + 1 < cuts.size(); ++i) {
    const int64_t d_begin = cuts[i], d_end = cuts[i + 1];
    if (d_end > d_begin) {
      const std::vector<int64_t> sub(off.begin() + d_begin, off.begin() + d_end + 1);
      const std::vector<int64_t> rr = make_ranges(sub, target);
      for (size_t j = 1; j < rr.size(); ++j) r.push_back(d_begin + rr[j]);
    }
    part_range.push_back((int64_t)r.size() - 1);
  }
  return r;
}

// Sequential-sweep parts (lda_set_warm_start, lda_set_sequential_sweeps),
// seen from a shard whose documents start at global token base + off[d]:
// the corpus [g0, g0 + gn) is cut into LDA_WARM_BLOCKS token-balanced blocks,
// and block b into `parts` pieces at the cumulative fractions cum[i] / Q
// (Q = LDA_SEQ_FRACTION_UNIT; cum[0] = 0, cum[parts] = Q): the cut at (b, i)
// is the first document starting at or after g0 + gn (b Q + cum[i]) / (B Q),
// and piece i of every block belongs to part i.  Every shard of a
// token-balanced sharding into up to LDA_WARM_BLOCKS shards therefore holds
// documents of every part (round 3 had cut P contiguous parts, so at G = 8,
// P = 4 only 2 of 8 GPUs sampled in each step).  runs[i] = part i's local
// document runs [d0, d1), in order.  Integer arithmetic, the product gn (b Q
// + cum) in 128 bits (B Q = 2^25.5: int64 would overflow past gn ~ 2^37): the
// oracle (Python integers) cuts the same documents at any corpus size.
std::vector<std::vector<std::pair<int64_t, int64_t>>> seq_part_runs(const std::vector<int64_t>& off,
                                                                    const std::vector<int64_t>& cum,
                                                                    int64_t base, int64_t g0, int64_t gn) {
  const int64_t D = (int64_t)off.size() - 1;
  const int parts = (int)cum.size() - 1;
  const int64_t B = LDA_WARM_BLOCKS, Q = LDA_SEQ_FRACTION_UNIT;
  std::vector<std::vector<std::pair<int64_t, int64_t>>> runs((size_t)parts);
  int64_t prev = 0;
  for (int64_t b = 0; b < B; ++b)
    for (int i = 0; i < parts; ++i) {
      int64_t next = D;
      if (b + 1 < B || i + 1 < parts) {
        const int64_t tgt = g0 + (int64_t)((__int128)gn * (b * Q + cum[(size_t)i + 1]) / (B * Q)) - base;
        next = std::lower_bound(off.begin(), off.end(), tgt) - off.begin();
        next = std::min(std::max(next, prev), D);
      }
      if (next > prev) runs[(size_t)i].push_back({prev, next});
      prev = next;
    }
  return runs;
}

// cumulative fractions of `parts` equal parts, in units of 1 / LDA_SEQ_FRACTION_UNIT (exact)
std::vector<int64_t> equal_cum(int parts) {
  std::vector<int64_t> cum((size_t)parts + 1);
  for (int i = 0; i <= parts; ++i) cum[(size_t)i] = (int64_t)LDA_SEQ_FRACTION_UNIT * i / parts;
  return cum;
}

// The work ranges of each part's document runs: ranges never cross a run
// end, and the last ~1/8 of a part's tokens go in quarter-size ranges (its
// launch tail).  Range r is documents [start[r], end[r]); part_range[i] is
// part i's first range.
void make_run_ranges(const std::vector<int64_t>& off, int64_t target,
                     const std::vector<std::vector<std::pair<int64_t, int64_t>>>& runs,
                     std::vector<int64_t>& start, std::vector<int64_t>& end,
                     std::vector<int64_t>& part_range) {
  start.clear();
  end.clear();
  part_range.assign(1, 0);
  const int64_t tail_target = std::max<int64_t>(16, target / 4);
  for (const auto& pr : runs) {
    int64_t total = 0;
    for (const auto& r : pr) total += off[r.second] - off[r.first];
    const int64_t tail_from = total / 8 * 7;
    int64_t seen = 0;
    for (const auto& r : pr) {
      int64_t s = r.first;
      for (int64_t d = r.first; d < r.second; ++d) {
        const int64_t tgt = seen >= tail_from ? tail_target : target;
        if (off[d + 1] - off[s] >= tgt || d + 1 == r.second) {
          seen += off[d + 1] - off[s];
          start.push_back(s);
          end.push_back(d + 1);
          s = d + 1;
        }
      }
    }
    part_range.push_back((int64_t)start.size());
  }
}

// A split sweep's ranges: the shard's own token-balanced cuts.  parts == 1
// gives exactly make_ranges(off, target).
std::vector<int64_t> make_part_ranges(const std::vector<int64_t>& off, int64_t target, int parts,
                                      std::vector<int64_t>& part_range) {
  const int64_t D = (int64_t)off.size() - 1;
  return make_cut_ranges(off, target, part_cuts(off, parts, 0, off[0], off[D] - off[0]), part_range);
}

template <typename T>
hipError_t dalloc(T** p, size_t n) {
  *p = nullptr;
  if (n == 0) n = 1;
  return hipMalloc(reinterpret_cast<void**>(p), n * sizeof(T));
}

}  // namespace

namespace lda_abi {
void set_error(const std::string& msg) { g_last_error = msg; }
void check_host_alloc() {
  if (g_fail_alloc > 0 && --g_fail_alloc == 0) throw std::bad_alloc();
}
}  // namespace lda_abi
using lda_abi::host_vector;

struct lda_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  int32_t K = 0, Kp = 0, C = 0, V = 0;
  int64_t D = 0, N = 0, R = 0;
  std::vector<double> alpha;
  double beta = 0.0;
  uint64_t seed = 0;
  int64_t token_base = 0;
  uint32_t sweep = 0;
  bool pending = true;
  int cus = 256;
  int sampler = LDA_SAMPLER_DENSE;
  int sample_blocks = 0, sample_blocks_frozen = 0, waves_per_block = 4;
  // sparse rows of the snapshot (LDA_SAMPLER_SPARSE)
  uint32_t* ent = nullptr;
  int64_t* row_off = nullptr;
  int32_t* row_nnz = nullptr;
  uint32_t* row_rnd = nullptr;   // row_off / 64: the large-K sampler's 32-bit row starts
  // the large-K sampler's ring depth (register rounds): 0 = the default,
  // lda::SB_RB_SHORT_ROUNDS = the short ring.  Both give the same draws; which
  // is faster depends on the rows' lengths, which shrink as the chain burns
  // in, so the context times them (big_rb_next): three consecutive sweeps'
  // first launches at default / short / default depth (a linear drift of the
  // sweep time cancels against the mean of the outer two), then the faster
  // is kept for PROBE_HOLD sweeps; a probe costs one sweep at the slower
  // depth and one host wait.  LDA_SB_RB=<n> at lda_create fixes the depth.
  static constexpr int64_t PROBE_HOLD = 16;
  // no probe in the context's first PROBE_FIRST sweeps: right after the
  // random start the rows shrink fastest and the drift is far from linear
  // (a probe over sweeps 0-2 picked the short ring, 3% slower there); the
  // default depth is the right one near init
  static constexpr int64_t PROBE_FIRST = 8;
  int64_t big_sweeps = 0;            // sweeps sampled by the large-K sampler
  bool big_rb_auto = true;
  int big_rb = 0;
  int big_probe = 0;                 // probe launches issued so far (0..3)
  int big_probe_slot = -1;           // the sweep being sampled is probe launch i (else -1)
  int64_t big_hold = 0;              // sweeps left before the next probe
  hipEvent_t big_ev[3][2] = {};
  // what probe i timed: the first non-empty launch of its sweep, tagged
  // (sweep kind, part, ranges); -1 = nothing launched (an empty shard or
  // part).  Probes are compared only when all three timed the same tag.
  int64_t big_ev_tag[3] = {-1, -1, -1};
  bool rows_ready = false;
  bool fused_apply = true;   // k_apply_build (LDA_FUSED_APPLY=0: k_apply_cols + k_build_sparse, A/B)
  int half = 0;    // dense K <= 128: 1 = the half-wave variant, 2 = the quarter-wave one (LDA_DENSE_HALF)
  // lda_infer: word totals of the snapshot (TopicInferencer's empty-row test),
  // valid while apply_gen == totals_gen, and grow-only scratch buffers, so a
  // one-document call (the reference's predict loop) costs no allocation and
  // no pass over nw
  uint64_t apply_gen = 0, totals_gen = ~0ull;
  std::vector<int32_t> word_totals;
  int32_t *inf_words = nullptr, *inf_z = nullptr, *inf_acc = nullptr, *inf_q = nullptr;
  int64_t *inf_doff = nullptr, *inf_range = nullptr;
  size_t inf_cap[6] = {};
  // 16-bit rows of the snapshot (LDA_SAMPLER_DENSE)
  uint16_t* nw16 = nullptr;
  uint8_t* wide = nullptr;
  int64_t tokens_per_range = 0;
  std::vector<int64_t> doc_off_h;
  std::vector<int64_t> ranges_h;   // host copy of range_doc
  // dense samplers' recount: the sampler writes only z, then
  // every word row of the shard is recounted from a word-sorted token index
  // into the exchange buffer, which then holds counts, not changes.  Which
  // sweeps recount: count_mode (LDA_COUNT_*) and, for AUTO, the first
  // recount_sweeps sweeps since the counts were (re)seeded.
  int count_mode = LDA_COUNT_AUTO;
  int32_t recount_sweeps = 0;
  int64_t sweeps_since_seed = 0;
  bool sweep_recount = false;      // the sweep being sampled recounts
  // the word-ordered copy of z for the quarter-wave sampler's recount sweeps
  // (zw[zpos[i]] = z[i] in the recount index's order; the sampler updates it,
  // the recount streams it).  Valid while every sweep since it was built kept
  // it current; rebuilt from z at a recount sweep otherwise.
  int32_t* zw = nullptr;
  uint32_t* zpos = nullptr;
  bool zw_valid = false;
  bool sweep_zw = false;           // the sweep being sampled keeps zw current
  bool use_zw = true;              // LDA_ZW=0: the recount gathers z through perm (A/B)
  bool pending_absolute = false;   // the pending buffer holds counts (recount) rather than a delta
  bool recount_ok = false;         // dense sampler, N < 2^32
  // warm start (lda_set_warm_start): sweeps with a sweep counter below
  // warm_sweeps run in warm_parts SEQUENTIAL parts (each applied before
  // the next part samples; all through buffer 0), over their own ranges
  // A sequential schedule: parts sampled in order, each applied before the
  // next samples (all through buffer 0), over their own work ranges
  struct SeqSchedule {
    int parts = 1;
    int64_t* range_doc = nullptr;    // range starts [R], then the ends (range_end)
    int64_t* range_end = nullptr;
    std::vector<int64_t> part_range{0, 0};
    std::vector<int64_t> cum{0, LDA_SEQ_FRACTION_UNIT};
  };
  SeqSchedule warm;                  // lda_set_warm_start: sweeps below warm_sweeps
  int32_t warm_sweeps = 0;
  SeqSchedule steady;                // lda_set_sequential_sweeps: every other sweep
  bool sweep_seq = false;            // the sweep being sampled is sequential ...
  int sweep_kind = 0;                // ... 1: a warm-start sweep, 2: a steady one
  uint32_t* perm = nullptr;        // [N] token indices grouped by (part, word)
  int32_t* items = nullptr;        // int4 {word, first perm index, tokens, split} per work item
  std::vector<int64_t> part_item{0, 0};
  int recount_blocks = 0;

  int32_t* words = nullptr;
  int32_t* z = nullptr;
  int64_t* doc_off = nullptr;
  int64_t* range_doc = nullptr;
  int32_t* queue = nullptr;
  int32_t* nw = nullptr;
  int32_t* nwsum = nullptr;
  int32_t* delta = nullptr;
  // split sweep (lda_set_exchange_parts): part i samples the work ranges
  // [part_range[i], part_range[i+1]) into delta_part[i] (delta_part[0] == delta)
  int parts = 1, next_part = 0, reserve_cus = 0;
  // compact exchange (lda_exchange_pack): per buffer slot, the packed words
  // [V*Kp/2 | Kp] and the escape list [1 + 3 cap], grow-only
  int32_t* exch_packed[LDA_MAX_EXCHANGE_PARTS] = {};
  int32_t* exch_esc[LDA_MAX_EXCHANGE_PARTS] = {};
  size_t exch_esc_cap[LDA_MAX_EXCHANGE_PARTS] = {};
  int32_t exch_cells = 2;          // cells per packed word: 2 (16-bit fields) or 4 (8-bit)
  int32_t* delta_part[LDA_MAX_EXCHANGE_PARTS] = {};
  std::vector<int64_t> part_range{0, 0};
  double* alpha_d = nullptr;
  float* alpha_f = nullptr;
  float* inv = nullptr;
  float* inv_m1 = nullptr;
  // the large-K sampler's per-sweep tables (k_big_tables; C >= 32 sparse only)
  lda::BigTables big{};
  double* partial = nullptr;
  unsigned long long* nonzero = nullptr;
  int partial_blocks = 1024;
  // lda_log_likelihood_enqueue / _collect: results in flight, each copied into
  // pinned host memory [doc partials | word partials | nonzero counts | nwsum]
  struct LLSlot {
    void* host = nullptr;
    hipEvent_t done = nullptr;
    int64_t ticket = -1;
    double alpha_sum = 0.0, beta = 0.0;
  };
  static constexpr int LL_SLOTS = 16;
  LLSlot ll[LL_SLOTS];
  int64_t ll_next = 0;
  // lda_doc_topic_histograms_accumulate / _take: alpha statistics summed on
  // the device over sampled sweeps [doc lengths (L+1) | topics K x (L+1)]
  int32_t* stat_buf = nullptr;
  int32_t stat_len = -1;
  // lda_count_histogram's device histogram, grow-only (an optimisation every
  // 20 sweeps of a small corpus had paid a hipMalloc + hipFree each time)
  int32_t* chist = nullptr;
  size_t chist_cap = 0;
  // lda_sweep's plain sweeps as hipGraphs of k x (sampler, apply), k <= 16:
  // one launch for k sweeps instead of ~6 runtime calls per sweep (the
  // reference's ~16k-token corpus is host-bound at ~45 us per sweep against
  // ~32 us of kernels).  The sweep counter is read by the sampler from
  // state_dev, which each apply advances, and beta from there too (the
  // optimisation changes it every few sweeps); graphs are rebuilt when a
  // captured argument changes (graph_key).
  static constexpr int GRAPH_MAX = 16;
  bool use_graphs = true;
  uint32_t* state_dev = nullptr;      // [0] sweep, [1] beta, [2] V*beta (fp32 bits)
  int64_t state_sweep = -1;           // the sweep state_dev[0] holds (-1: unknown)
  bool state_beta = false;            // state_dev[1..2] hold the current beta
  // lda_set_alpha_beta's upload source (pinned, so the copy is asynchronous;
  // the event guards its reuse) and lda_hyper_statistics' staging
  double* alpha_pin = nullptr;
  hipEvent_t alpha_ev = nullptr;
  bool alpha_ev_live = false;
  int32_t* hyper_pin = nullptr;
  size_t hyper_pin_cap = 0;
  hipGraphExec_t graphs[GRAPH_MAX + 1] = {};
  hipEvent_t graph_ev = nullptr;      // recorded after each graph launch
  hipEvent_t switch_ev = nullptr;     // lda_set_stream: orders the new stream after the old
  bool graph_ev_live = false;
  struct GraphKey {
    const void* range_doc = nullptr;
    int64_t R = -1;
    hipStream_t stream = nullptr;
    const void* seq = nullptr;         // steady sequential sweeps: their ranges (else null)
    int seq_parts = 0;
    bool operator==(const GraphKey& o) const {
      return range_doc == o.range_doc && R == o.R && stream == o.stream && seq == o.seq &&
             seq_parts == o.seq_parts;
    }
  } graph_key;
  // event pairs around the last LDA_TIME_RING sampler launches (lda_sample_times)
  static constexpr int LDA_TIME_RING = 256;
  hipEvent_t ev0[LDA_TIME_RING] = {}, ev1[LDA_TIME_RING] = {}, ev2[LDA_TIME_RING] = {};
  bool recounted[LDA_TIME_RING] = {};   // the launch in this slot ran the recount (ev1 -> ev2)
  int64_t launches = 0;

  ~lda_ctx() {
    if (device >= 0) (void)hipSetDevice(device);
    // work still queued (graph sweeps, asynchronous uploads and read-backs)
    // finishes before its buffers, graphs and pinned staging are released
    if (device >= 0) (void)hipDeviceSynchronize();
    for (void* p : {(void*)words, (void*)z, (void*)doc_off, (void*)range_doc, (void*)queue,
                    (void*)nw, (void*)nwsum, (void*)delta, (void*)alpha_d, (void*)alpha_f,
                    (void*)inv, (void*)inv_m1, (void*)partial, (void*)nonzero, (void*)ent,
                    (void*)row_off, (void*)row_nnz, (void*)row_rnd, (void*)nw16, (void*)wide, (void*)inf_words,
                    (void*)inf_z, (void*)inf_acc, (void*)inf_q, (void*)inf_doff, (void*)inf_range,
                    (void*)perm, (void*)items, (void*)warm.range_doc, (void*)steady.range_doc,
                    (void*)big.tab, (void*)big.tab_m1, (void*)big.F, (void*)big.pfx, (void*)big.scal})
      if (p) (void)hipFree(p);
    for (int i = 1; i < LDA_MAX_EXCHANGE_PARTS; ++i)
      if (delta_part[i]) (void)hipFree(delta_part[i]);
    for (int i = 0; i < LDA_MAX_EXCHANGE_PARTS; ++i) {
      if (exch_packed[i]) (void)hipFree(exch_packed[i]);
      if (exch_esc[i]) (void)hipFree(exch_esc[i]);
    }
    for (auto& sl : ll) {
      if (sl.done) (void)hipEventSynchronize(sl.done);
      if (sl.host) (void)hipHostFree(sl.host);
      if (sl.done) (void)hipEventDestroy(sl.done);
    }
    if (stat_buf) (void)hipFree(stat_buf);
    if (chist) (void)hipFree(chist);
    for (auto& g : graphs)
      if (g) (void)hipGraphExecDestroy(g);
    if (graph_ev) (void)hipEventDestroy(graph_ev);
    for (auto& e : big_ev)
      for (hipEvent_t x : e)
        if (x) (void)hipEventDestroy(x);
    if (switch_ev) (void)hipEventDestroy(switch_ev);
    if (state_dev) (void)hipFree(state_dev);
    if (zw) (void)hipFree(zw);
    if (zpos) (void)hipFree(zpos);
    if (alpha_pin) (void)hipHostFree(alpha_pin);
    if (alpha_ev) (void)hipEventDestroy(alpha_ev);
    if (hyper_pin) (void)hipHostFree(hyper_pin);
    for (int i = 0; i < LDA_TIME_RING; ++i) {
      if (ev0[i]) (void)hipEventDestroy(ev0[i]);
      if (ev1[i]) (void)hipEventDestroy(ev1[i]);
      if (ev2[i]) (void)hipEventDestroy(ev2[i]);
    }
    if (own_stream) (void)hipStreamDestroy(own_stream);
  }

  lda::SampleParams params(bool frozen) const {
    lda::SampleParams p{};
    p.words = words;
    p.z = z;
    p.doc_off = doc_off;
    p.range_doc = range_doc;
    p.range_end = range_doc + 1;     // contiguous ranges: range r ends where r + 1 starts
    p.num_ranges = R;
    p.queue = queue;
    p.nw = nw;
    p.delta = delta;
    p.dsum = delta + (int64_t)V * Kp;
    p.alpha = alpha_f;
    p.inv = inv;
    p.inv_m1 = inv_m1;
    p.beta = (float)beta;
    p.K = K;
    p.token_base = token_base;
    p.k0 = (uint32_t)seed;
    p.k1 = (uint32_t)(seed >> 32);
    p.c2 = sweep;
    p.c3 = lda::STREAM_SAMPLE;
    p.ent = ent;
    p.row_off = row_off;
    p.row_nnz = row_nnz;
    p.row_rnd = row_rnd;
    p.nw16 = nw16;
    p.wide = wide;
    p.big = big;
    (void)frozen;
    return p;
  }
};

// Sparse-row capacities: min(Kp, total count of the word) rounded up to whole
// 64-entry rounds, fixed once the global counts exist (word totals never
// change afterwards).
static lda_status build_row_capacity(lda_ctx* c) {
  int32_t* caps = nullptr;
  HIP_TRY(dalloc(&caps, c->V));
  std::vector<int32_t> h(c->V);
  hipError_t e = lda::launch_row_caps(c->nw, c->V, c->Kp, caps, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), caps, sizeof(int32_t) * c->V, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(caps);
  HIP_TRY(e);
  std::vector<int64_t> off(c->V + 1);
  off[0] = 0;
  // whole rounds of 64 entries (k_build_sparse zero-fills the padding)
  for (int w = 0; w < c->V; ++w) off[w + 1] = off[w] + ((h[w] + 63) & ~int64_t(63));
  // the large-K sampler reads a row's start as a 32-bit count of whole
  // rounds: 2^32 rounds are 2^38 entries (1 TiB), beyond any device memory
  std::vector<uint32_t> rnd(c->V);
  for (int w = 0; w < c->V; ++w) rnd[w] = (uint32_t)(off[w] >> 6);
  HIP_TRY(dalloc(&c->row_off, c->V + 1));
  HIP_TRY(dalloc(&c->row_nnz, c->V));
  HIP_TRY(dalloc(&c->row_rnd, c->V));
  HIP_TRY(dalloc(&c->ent, (size_t)off[c->V]));
  HIP_TRY(hipMemcpyAsync(c->row_off, off.data(), sizeof(int64_t) * (c->V + 1), hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->row_rnd, rnd.data(), sizeof(uint32_t) * c->V, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->rows_ready = true;
  return LDA_OK;
}

// The recount's word-sorted token index for the current exchange parts:
// tokens per (part, word) on the GPU, offsets and work items on the host
// (words of more than RECOUNT_ITEM_TOKENS tokens in a part are split; each
// part's items longest first, so the work queue ends on short ones), then
// the scatter of token indices.  Words never change, so this runs at create
// and when the parts change.
static lda_status build_recount_index(lda_ctx* c) {
  if (c->perm) (void)hipFree(c->perm);
  if (c->items) (void)hipFree(c->items);
  c->perm = nullptr;
  c->items = nullptr;
  c->part_item.assign((size_t)c->parts + 1, 0);
  c->zw_valid = false;             // zw follows perm's order
  if (!c->recount_ok || c->N == 0) return LDA_OK;
  lda::PartSpans ps{};
  ps.parts = c->parts;
  for (int i = 0; i <= c->parts; ++i)
    ps.tok[i] = c->doc_off_h[(size_t)c->ranges_h[(size_t)c->part_range[(size_t)i]]];
  const size_t cells = (size_t)c->parts * (size_t)c->V;
  uint32_t* cnt = nullptr;
  HIP_TRY(dalloc(&cnt, cells));
  std::vector<uint32_t> h(cells);
  hipError_t e = hipMemsetAsync(cnt, 0, sizeof(uint32_t) * cells, c->stream);
  if (e == hipSuccess) e = lda::launch_word_hist(c->words, c->N, ps, c->V, cnt, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), cnt, sizeof(uint32_t) * cells, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    (void)hipFree(cnt);
    HIP_TRY(e);
  }
  std::vector<int32_t> it;
  uint32_t off = 0;
  const uint32_t S = (uint32_t)lda::RECOUNT_ITEM_TOKENS;
  for (int pt = 0; pt < c->parts; ++pt) {
    const size_t first = it.size() / 4;
    for (int32_t w = 0; w < c->V; ++w) {
      const uint32_t n = h[(size_t)pt * c->V + w];
      h[(size_t)pt * c->V + w] = off;   // becomes the scatter cursor
      for (uint32_t b = 0; b < n; b += S)
        it.insert(it.end(), {w, (int32_t)(off + b), (int32_t)std::min(S, n - b), n > S ? 1 : 0});
      off += n;
    }
    // longest items first within the part (stable: ties keep word order)
    std::vector<size_t> order(it.size() / 4 - first);
    for (size_t j = 0; j < order.size(); ++j) order[j] = first + j;
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return it[4 * a + 2] > it[4 * b + 2]; });
    std::vector<int32_t> sorted;
    sorted.reserve(order.size() * 4);
    for (size_t j : order) sorted.insert(sorted.end(), it.begin() + 4 * j, it.begin() + 4 * j + 4);
    std::copy(sorted.begin(), sorted.end(), it.begin() + 4 * first);
    c->part_item[(size_t)pt + 1] = (int64_t)(it.size() / 4);
  }
  e = dalloc(&c->perm, (size_t)c->N);
  if (e == hipSuccess) e = dalloc(&c->items, std::max<size_t>(it.size(), 4));
  if (e == hipSuccess) e = hipMemcpyAsync(cnt, h.data(), sizeof(uint32_t) * cells, hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = lda::launch_word_scatter(c->words, c->N, ps, c->V, cnt, c->perm, c->stream);
  if (e == hipSuccess && !it.empty())
    e = hipMemcpyAsync(c->items, it.data(), sizeof(int32_t) * it.size(), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(cnt);
  HIP_TRY(e);
  return LDA_OK;
}

// nwsum += its pending delta and the per-topic tables (k_prepare_topics),
// then the large-K sampler's fixed-point tables from them
static hipError_t prepare_tables(lda_ctx* c) {
  hipError_t e = lda::launch_prepare_topics(c->nwsum, c->delta + (int64_t)c->V * c->Kp, c->alpha_d, c->beta,
                                            (double)c->V * c->beta, c->K, c->Kp, c->alpha_f, c->inv,
                                            c->inv_m1, c->stream);
  if (e == hipSuccess && c->big.tab)
    e = lda::launch_big_tables(c->nwsum, c->alpha_f, c->inv, c->inv_m1, c->K, c->Kp, (float)c->beta, c->big,
                               c->stream);
  return e;
}

static lda_status apply_impl(lda_ctx* c) {
  if (c->next_part != 0 && !c->sweep_seq)
    return fail(LDA_ERR_STATE, "lda_apply inside a split sweep: sample every part first");
  c->apply_gen++;
  HIP_TRY(hipSetDevice(c->device));
  // a split sweep's later parts are folded into part 0's buffer (the one the
  // apply kernels read) and zeroed; a warm-start sweep's parts all use buffer 0
  if (!c->sweep_seq)
    for (int i = 1; i < c->parts; ++i)
      HIP_TRY(lda::launch_fold_delta(c->delta, c->delta_part[i], (int64_t)c->V * c->Kp + c->Kp, c->stream));
  if (c->sampler == LDA_SAMPLER_DENSE) {
    // one launch: apply, 16-bit rows, topic tables, queue reset (k_apply_packed)
    lda::TopicTables t{c->nwsum, c->alpha_d, c->alpha_f, c->inv, c->inv_m1,
                       (float)((double)c->V * c->beta), c->K, c->queue, c->pending_absolute ? 1 : 0};
    HIP_TRY(lda::launch_apply_packed(c->nw, c->delta, c->V, c->Kp, c->nw16, c->wide, t, c->stream));
    c->pending = false;
    return LDA_OK;
  }
  // the sparse samplers write no nwsum delta: k_apply_cols derives it from the
  // (summed) nw delta's column sums.  Whatever the nwsum cells hold (the
  // initial counts of k_count, an exchange's sum) is the same column sum, so
  // it is dropped and recomputed
  HIP_TRY(hipMemsetAsync(c->delta + (int64_t)c->V * c->Kp, 0, sizeof(int32_t) * c->Kp, c->stream));
  if (c->sampler == LDA_SAMPLER_SPARSE && c->rows_ready && c->fused_apply) {
    // one pass: apply, column sums, sparse rows (k_apply_build); then the
    // topic tables from the column sums
    HIP_TRY(lda::launch_apply_build(c->nw, c->delta, c->V, c->Kp, c->row_off, c->ent, c->row_nnz,
                                    c->delta + (int64_t)c->V * c->Kp, c->stream));
    HIP_TRY(prepare_tables(c));
    c->pending = false;
    return LDA_OK;
  }
  HIP_TRY(lda::launch_apply_cols(c->nw, c->delta, c->V, c->Kp, c->delta + (int64_t)c->V * c->Kp, c->stream));
  HIP_TRY(prepare_tables(c));
  if (c->sampler == LDA_SAMPLER_SPARSE) {
    if (!c->rows_ready) {
      lda_status s = build_row_capacity(c);
      if (s) return s;
    }
    HIP_TRY(lda::launch_build_sparse(c->nw, c->V, c->Kp, c->row_off, c->ent, c->row_nnz, c->stream));
  } else {
    HIP_TRY(lda::launch_build_packed(c->nw, c->V, c->Kp, c->nw16, c->wide, c->stream));
  }
  c->pending = false;
  return LDA_OK;
}

// Is the next sweep a warm-start sweep (sequential parts)?
// (keyed by the sweep counter, which a resumed model carries: estimate(15) +
// estimate(25) runs the same warm start as estimate(40))
static int next_sweep_kind(const lda_ctx* c) {
  if (c->warm.parts > 1 && (int64_t)c->sweep < (int64_t)c->warm_sweeps) return 1;
  return c->steady.parts > 1 ? 2 : 0;
}
static bool next_sweep_sequential(const lda_ctx* c) { return next_sweep_kind(c) != 0; }
// the schedule of the sweep in progress (or of the next one)
static const lda_ctx::SeqSchedule& seq_schedule(const lda_ctx* c) {
  const int kind = c->next_part != 0 ? c->sweep_kind : next_sweep_kind(c);
  return kind == 1 ? c->warm : c->steady;
}
// Parts of the sweep in progress, or of the next one
static int sweep_parts(const lda_ctx* c) {
  const bool seq = c->next_part != 0 ? c->sweep_seq : next_sweep_sequential(c);
  return seq ? seq_schedule(c).parts : c->parts;
}

// Will the next sweep recount?  A sequential sweep (warm start, staleness)
// recounts the WHOLE shard after each of its parts (the parts are applied one
// by one, and absolute counts must include every token), so its recount
// costs a full pass per part: AUTO keeps it to plain sweeps (its measured
// crossover), LDA_COUNT_RECOUNT makes every sweep recount.
static bool next_sweep_recounts(const lda_ctx* c) {
  if (!c->recount_ok) return false;
  if (c->count_mode == LDA_COUNT_RECOUNT) return true;
  if (c->count_mode == LDA_COUNT_DELTA || next_sweep_sequential(c)) return false;
  return c->sweeps_since_seed < c->recount_sweeps;
}

static lda_status reseed_counts(lda_ctx* c) {
  // local (word, topic) counts of this shard become the pending delta
  for (int i = 0; i < c->parts; ++i)
    HIP_TRY(hipMemsetAsync(c->delta_part[i], 0, sizeof(int32_t) * ((size_t)c->V * c->Kp + c->Kp), c->stream));
  c->next_part = 0;
  HIP_TRY(hipMemsetAsync(c->nw, 0, sizeof(int32_t) * (size_t)c->V * c->Kp, c->stream));
  HIP_TRY(hipMemsetAsync(c->nwsum, 0, sizeof(int32_t) * c->Kp, c->stream));
  HIP_TRY(lda::launch_count(c->words, c->z, c->N, c->Kp, c->delta, c->delta + (int64_t)c->V * c->Kp,
                            c->stream));
  c->pending = true;
  c->pending_absolute = false;   // nw is zero: adding the local counts sets them
  c->sweeps_since_seed = 0;
  c->zw_valid = false;           // z may have been replaced
  return LDA_OK;
}

extern "C" {

const char* lda_last_error(void) { return g_last_error.c_str(); }
void lda_debug_fail_host_alloc(int32_t nth) { g_fail_alloc = nth > 0 ? nth : 0; }
#define LDA_STR2(x) #x
#define LDA_STR(x) LDA_STR2(x)
// the version string carries the header's ABI number (they had drifted apart)
const char* lda_version(void) { return "lda_mi355x 0.4.0 (gfx950; ABI " LDA_STR(LDA_ABI_VERSION) ")"; }
int32_t lda_abi_version(void) { return LDA_ABI_VERSION; }
int32_t lda_padded_topics(int32_t num_topics) { return pad_topics(num_topics); }

lda_status lda_create(lda_ctx** out, const lda_config* cfg, const int64_t* doc_off,
                      const int32_t* words, const int32_t* z_init) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!out || !cfg || !doc_off) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *out = nullptr;
  if (cfg->num_topics < 1) return fail(LDA_ERR_INVALID_ARG, "num_topics must be >= 1");
  if (cfg->num_topics > LDA_MAX_TOPICS)
    return fail(LDA_ERR_UNSUPPORTED, "num_topics above LDA_MAX_TOPICS (4096)");
  if (cfg->num_topics > LDA_MAX_TOPICS_DENSE && cfg->sampler == LDA_SAMPLER_DENSE)
    return fail(LDA_ERR_UNSUPPORTED,
                "num_topics above LDA_MAX_TOPICS_DENSE (1024): use LDA_SAMPLER_SPARSE");
  if (cfg->num_types < 1) return fail(LDA_ERR_INVALID_ARG, "num_types must be >= 1");
  // the dense sampler indexes nw cells with 32 bits
  if (cfg->sampler == LDA_SAMPLER_DENSE &&
      (int64_t)cfg->num_types * pad_topics(cfg->num_topics) >= (int64_t(1) << 32))
    return fail(LDA_ERR_UNSUPPORTED, "num_types * padded topics >= 2^32 with the dense sampler: use LDA_SAMPLER_SPARSE");
  if (cfg->num_docs < 0) return fail(LDA_ERR_INVALID_ARG, "num_docs must be >= 0");
  if (!cfg->alpha) return fail(LDA_ERR_INVALID_ARG, "alpha is null");
  if (!(cfg->beta > 0.0)) return fail(LDA_ERR_INVALID_ARG, "beta must be > 0");
  if (cfg->sampler != LDA_SAMPLER_DENSE && cfg->sampler != LDA_SAMPLER_SPARSE)
    return fail(LDA_ERR_INVALID_ARG, "sampler must be LDA_SAMPLER_DENSE or LDA_SAMPLER_SPARSE");
  for (int k = 0; k < cfg->num_topics; ++k)
    if (!(cfg->alpha[k] > 0.0)) return fail(LDA_ERR_INVALID_ARG, "alpha must be > 0");
  const int64_t D = cfg->num_docs;
  std::vector<int64_t> off = host_vector<int64_t>((size_t)D + 1);
  for (int64_t d = 0; d <= D; ++d) {
    off[d] = doc_off[d] - doc_off[0];
    if (d > 0 && off[d] < off[d - 1]) return fail(LDA_ERR_INVALID_ARG, "doc_off not monotone");
  }
  const int64_t N = off[D];
  if (N > 0 && !words) return fail(LDA_ERR_INVALID_ARG, "words is null");
  if (pad_topics(cfg->num_topics) > 1024)
    for (int64_t d = 0; d < D; ++d)
      if (off[d + 1] - off[d] > LDA_MAX_DOC_TOKENS_BIGK)
        return fail(LDA_ERR_UNSUPPORTED, "document longer than 65535 tokens with num_topics > 1024");
  for (int64_t i = 0; i < N; ++i)
    if (words[i] < 0 || words[i] >= cfg->num_types)
      return fail(LDA_ERR_INVALID_ARG, "word id out of range [0, V)");
  if (z_init)
    for (int64_t i = 0; i < N; ++i)
      if (z_init[i] < 0 || z_init[i] >= cfg->num_topics)
        return fail(LDA_ERR_INVALID_ARG, "z_init topic out of range [0, K)");

  lda_ctx* c = new (std::nothrow) lda_ctx();
  if (!c) return fail(LDA_ERR_OUT_OF_MEMORY, "host allocation");
  c->device = cfg->device;
  c->sampler = cfg->sampler;
  c->K = cfg->num_topics;
  c->Kp = pad_topics(c->K);
  c->C = c->Kp / 64;
  c->V = cfg->num_types;
  c->D = D;
  c->N = N;
  c->alpha.assign(cfg->alpha, cfg->alpha + c->K);
  c->beta = cfg->beta;
  c->seed = cfg->seed;
  c->token_base = cfg->token_base;
  c->doc_off_h = off;

  auto bail = [&](lda_status s) {
    delete c;
    return s;
  };
#define CT(expr)                                    \
  do {                                              \
    hipError_t e_ = (expr);                         \
    if (e_ != hipSuccess)                           \
      return bail(fail(e_ == hipErrorOutOfMemory ? LDA_ERR_OUT_OF_MEMORY : LDA_ERR_DEVICE, \
                       std::string(#expr) + ": " + hipGetErrorString(e_)));               \
  } while (0)

  CT(hipSetDevice(c->device));
  CT(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
  c->stream = c->own_stream;
  hipDeviceProp_t prop;
  CT(hipGetDeviceProperties(&prop, c->device));
  c->cus = prop.multiProcessorCount;
  if (c->sampler == LDA_SAMPLER_SPARSE) {
    c->sample_blocks = lda::sample_sparse_blocks_per_cu(c->C, false) * c->cus;
    c->sample_blocks_frozen = lda::sample_sparse_blocks_per_cu(c->C, true) * c->cus;
  } else {
    // K <= 128: the quarter-wave kernel (four documents per wave, oracle
    // exact_draw_quarter) by default -- C2 1.37x near init, 1.69x after
    // burn-in over k_sample<2>.  LDA_DENSE_HALF=0 selects the
    // full-wave k_sample<C>, =1 the half-wave variant (slower; kept for A/B).
    const char* hv = std::getenv("LDA_DENSE_HALF");
    const int want = (hv && hv[0] >= '0' && hv[0] <= '2') ? hv[0] - '0' : 2;
    c->half = c->C <= 2 ? want : 0;
    c->sample_blocks = lda::sample_blocks_per_cu(c->C, false, c->K, c->half) * c->cus;
    c->sample_blocks_frozen = lda::sample_blocks_per_cu(c->C, true, c->K, c->half) * c->cus;
  }
  c->waves_per_block = lda::sample_waves_per_block(c->C, c->sampler == LDA_SAMPLER_SPARSE, c->half);
  {
    // the dense samplers can recount (a uint32 index: < 2^32 tokens).  AUTO
    // recounts the first LDA_RECOUNT_SWEEPS_DEFAULT sweeps of a K <= 128
    // shard whose z fits the 256 MB Infinity Cache: C2 1.64 -> 1.46 ms per
    // sweep at sweep 3, 1.50 -> 1.36 at sweep 17, a loss by sweep 30 (1.03 ->
    // 1.36); at K = 1024 (C3) the atomics cost no more than the recount, and
    // C4's 1 GB z makes its gathers cost more than the atomics they replace
    // (profiles/r03/crossover/).  LDA_RECOUNT=0 / 1 forces the
    // delta / recount mode (A/B runs).
    c->recount_ok = c->sampler == LDA_SAMPLER_DENSE && N < (int64_t(1) << 32);
    // (and not for a small corpus: its few atomics cost less than a launch)
    c->recount_sweeps = c->recount_ok && c->Kp <= 128 && N >= (int64_t(1) << 20) &&
                                N * 4 <= (int64_t(256) << 20)
                            ? LDA_RECOUNT_SWEEPS_DEFAULT : 0;
    const char* rv = std::getenv("LDA_RECOUNT");
    if (rv && rv[0] == '0') c->count_mode = LDA_COUNT_DELTA;
    if (rv && rv[0] == '1') c->count_mode = LDA_COUNT_RECOUNT;
    c->recount_blocks = 8 * c->cus;
  }
  const int64_t waves = (int64_t)c->sample_blocks * c->waves_per_block;
  int64_t tpr = cfg->tokens_per_range;
  // ~32 ranges per wave: fine enough that the launch tail stays short (C4: +5%
  // over 8 per wave), coarse enough to amortise a range start; at least 16
  // tokens, so a small corpus spreads over many waves (C1, 16k tokens: 168 ->
  // 56 us per sweep against a 256-token floor)
  if (tpr <= 0) tpr = std::max<int64_t>(16, std::min<int64_t>(65536, N / std::max<int64_t>(1, waves * 32)));
  c->tokens_per_range = tpr;
  std::vector<int64_t> ranges = make_part_ranges(off, tpr, 1, c->part_range);
  c->R = (int64_t)ranges.size() - 1;
  c->ranges_h = ranges;

  CT(dalloc(&c->words, N));
  CT(dalloc(&c->z, N));
  CT(dalloc(&c->doc_off, D + 1));
  CT(dalloc(&c->range_doc, ranges.size()));
  CT(dalloc(&c->queue, LDA_MAX_EXCHANGE_PARTS));
  CT(dalloc(&c->nw, (size_t)c->V * c->Kp));
  CT(dalloc(&c->nwsum, c->Kp));
  if (c->sampler == LDA_SAMPLER_DENSE) {
    CT(dalloc(&c->nw16, (size_t)c->V * c->Kp));
    CT(dalloc(&c->wide, (size_t)c->V));
  }
  CT(dalloc(&c->delta, (size_t)c->V * c->Kp + c->Kp));
  c->delta_part[0] = c->delta;
  CT(dalloc(&c->alpha_d, c->K));
  CT(dalloc(&c->alpha_f, c->Kp));
  CT(dalloc(&c->inv, c->Kp));
  CT(dalloc(&c->inv_m1, c->Kp));
  if (c->sampler == LDA_SAMPLER_SPARSE && c->C >= 32) {
    CT(dalloc(&c->big.tab, c->Kp));
    CT(dalloc(&c->big.tab_m1, c->Kp));
    CT(dalloc(&c->big.F, c->Kp));
    CT(dalloc(&c->big.pfx, c->Kp));
    CT(dalloc(&c->big.scal, 1));
  }
  CT(dalloc(&c->partial, c->partial_blocks));
  CT(dalloc(&c->state_dev, 4));
  {
    const char* gv = std::getenv("LDA_GRAPHS");
    c->use_graphs = !(gv && gv[0] == '0');
    const char* fav = std::getenv("LDA_FUSED_APPLY");
    c->fused_apply = !(fav && fav[0] == '0');
    // LDA_SB_RB=short (or the short ring's rounds) / default (or any other
    // number): the large-K ring fixed instead of timed
    const char* rbv = std::getenv("LDA_SB_RB");
    if (rbv && rbv[0]) {
      c->big_rb_auto = false;
      const bool shrt = std::strcmp(rbv, "short") == 0 || std::atoi(rbv) == lda::SB_RB_SHORT_ROUNDS;
      c->big_rb = shrt ? lda::SB_RB_SHORT_ROUNDS : 0;
    }
    const char* zv = std::getenv("LDA_ZW");
    c->use_zw = !(zv && zv[0] == '0');
  }
  CT(dalloc(&c->nonzero, c->partial_blocks));
  for (int i = 0; i < lda_ctx::LDA_TIME_RING; ++i) {
    CT(hipEventCreate(&c->ev0[i]));
    CT(hipEventCreate(&c->ev1[i]));
    CT(hipEventCreate(&c->ev2[i]));
  }
  CT(hipMemsetAsync(c->queue, 0, sizeof(int32_t) * LDA_MAX_EXCHANGE_PARTS, c->stream));

  if (N > 0) CT(hipMemcpyAsync(c->words, words, sizeof(int32_t) * N, hipMemcpyHostToDevice, c->stream));
  CT(hipMemcpyAsync(c->doc_off, off.data(), sizeof(int64_t) * (D + 1), hipMemcpyHostToDevice, c->stream));
  CT(hipMemcpyAsync(c->range_doc, ranges.data(), sizeof(int64_t) * ranges.size(),
                    hipMemcpyHostToDevice, c->stream));
  CT(hipMemcpyAsync(c->alpha_d, c->alpha.data(), sizeof(double) * c->K, hipMemcpyHostToDevice, c->stream));
  if (z_init) {
    if (N > 0) CT(hipMemcpyAsync(c->z, z_init, sizeof(int32_t) * N, hipMemcpyHostToDevice, c->stream));
  } else {
    CT(lda::launch_init_z(c->z, N, c->K, c->token_base, (uint32_t)c->seed,
                          (uint32_t)(c->seed >> 32), c->stream));
  }
  {
    lda_status s = reseed_counts(c);
    if (s == LDA_OK && (c->recount_sweeps > 0 || c->count_mode == LDA_COUNT_RECOUNT))
      s = build_recount_index(c);
    if (s != LDA_OK) return bail(s);
  }
  CT(hipMemsetAsync(c->alpha_f, 0, sizeof(float) * c->Kp, c->stream));
  CT(hipStreamSynchronize(c->stream));
#undef CT
  *out = c;
  return LDA_OK;
  });
}

void lda_destroy(lda_ctx* ctx) { delete ctx; }

lda_status lda_set_stream(lda_ctx* c, void* s) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  hipStream_t ns = s ? (hipStream_t)s : c->own_stream;
  if (ns != c->stream) {
    // work already queued on the old stream comes first on the new one,
    // without a host wait (the caller need not synchronize to switch)
    HIP_TRY(hipSetDevice(c->device));
    if (!c->switch_ev) HIP_TRY(hipEventCreateWithFlags(&c->switch_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->switch_ev, c->stream));
    HIP_TRY(hipStreamWaitEvent(ns, c->switch_ev, 0));
  }
  c->stream = ns;
  return LDA_OK;
  });
}

lda_status lda_get_stream(lda_ctx* c, void** s) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !s) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *s = (void*)c->stream;
  return LDA_OK;
  });
}

lda_status lda_synchronize(lda_ctx* c) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LDA_OK;
  });
}

lda_status lda_get_sweep(lda_ctx* c, uint32_t* s) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !s) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *s = c->sweep;
  return LDA_OK;
  });
}

lda_status lda_set_sweep(lda_ctx* c, uint32_t s) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  c->sweep = s;
  return LDA_OK;
  });
}

lda_status lda_get_shape(lda_ctx* c, int32_t* K, int32_t* Kp, int32_t* V, int64_t* D, int64_t* N) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (K) *K = c->K;
  if (Kp) *Kp = c->Kp;
  if (V) *V = c->V;
  if (D) *D = c->D;
  if (N) *N = c->N;
  return LDA_OK;
  });
}

lda_status lda_apply(lda_ctx* c) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  return apply_impl(c);
  });
}

// The large-K sampler's ring depth for the sweep about to be sampled (see
// lda_ctx::big_rb).  The first PROBE_FIRST sweeps take the default depth;
// big_hold > 0: holding, a sweep counts it down; then
// three probe launches (the sweeps' first parts) at default / short / default
// depth; the sweep after them waits for the third (one host wait per probe:
// a read-back that lagged the host's queue would choose by the rows of many
// sweeps ago) and keeps the faster depth for the next PROBE_HOLD sweeps.
static lda_status big_rb_next(lda_ctx* c) {
  c->big_probe_slot = -1;
  if (c->big_sweeps++ < lda_ctx::PROBE_FIRST) {
    c->big_rb = 0;
    return LDA_OK;
  }
  if (c->big_hold > 0) {
    --c->big_hold;
    return LDA_OK;
  }
  if (c->big_probe < 3) {                       // the next probe launch
    if (!c->big_ev[0][0])
      for (auto& e : c->big_ev)
        for (hipEvent_t& x : e) HIP_TRY(hipEventCreate(&x));
    c->big_rb = c->big_probe == 1 ? lda::SB_RB_SHORT_ROUNDS : 0;
    c->big_ev_tag[c->big_probe] = -1;
    c->big_probe_slot = c->big_probe++;
    return LDA_OK;
  }
  // decide only when the three probes timed the same launch shape (a probe
  // whose sweep launched nothing, or that straddled a schedule change, is no
  // comparison): otherwise keep the default depth for a hold and retry
  const int64_t* t = c->big_ev_tag;
  if (t[0] >= 0 && t[0] == t[1] && t[1] == t[2]) {
    HIP_TRY(hipEventSynchronize(c->big_ev[2][1]));
    float ms[3];
    for (int i = 0; i < 3; ++i) HIP_TRY(hipEventElapsedTime(&ms[i], c->big_ev[i][0], c->big_ev[i][1]));
    c->big_rb = ms[1] < 0.5f * (ms[0] + ms[2]) ? lda::SB_RB_SHORT_ROUNDS : 0;
  } else {
    c->big_rb = 0;
  }
  c->big_hold = lda_ctx::PROBE_HOLD;
  c->big_probe = 0;
  return LDA_OK;
}

// One launch of the sampler over part `part` of a (possibly split) sweep.
static lda_status sample_part_impl(lda_ctx* c, int part) {
  if (part != c->next_part)
    return fail(LDA_ERR_STATE, "split sweep parts must be sampled in order 0, 1, ...");
  if (c->pending && (part == 0 || c->sweep_seq))
    return fail(LDA_ERR_STATE, part == 0 ? "lda_sample with a pending delta: call lda_apply first"
                                         : "warm-start sweep: apply each part before sampling the next");
  HIP_TRY(hipSetDevice(c->device));
  if (part == 0) {
    c->sweep_kind = next_sweep_kind(c);
    c->sweep_seq = c->sweep_kind != 0;
    if (c->sampler == LDA_SAMPLER_SPARSE && c->C >= 32 && c->big_rb_auto) {
      lda_status s = big_rb_next(c);
      if (s) return s;
    }
    c->sweep_recount = next_sweep_recounts(c);
    if (c->sweep_recount && !c->perm && c->N > 0) {
      lda_status s = build_recount_index(c);
      if (s) return s;
    }
    // the quarter-wave sampler keeps the word-ordered z copy current on a
    // recount sweep (the others leave it stale); built from z when stale
    c->sweep_zw = c->sweep_recount && c->use_zw && c->sampler == LDA_SAMPLER_DENSE && c->half == 2 && c->perm;
    if (c->sweep_zw && !c->zw_valid) {
      if (!c->zw) HIP_TRY(dalloc(&c->zw, (size_t)c->N));
      if (!c->zpos) HIP_TRY(dalloc(&c->zpos, (size_t)c->N));
      HIP_TRY(lda::launch_zw_build(c->perm, c->N, c->z, c->zpos, c->zw, c->stream));
    }
    c->zw_valid = c->sweep_zw;
  }
  const bool seq = c->sweep_seq;
  const lda_ctx::SeqSchedule& sch = c->sweep_kind == 1 ? c->warm : c->steady;
  const int nparts = seq ? sch.parts : c->parts;
  const std::vector<int64_t>& prange = seq ? sch.part_range : c->part_range;
  const int64_t r0 = prange[(size_t)part], r1 = prange[(size_t)part + 1];
  int32_t* buf = c->delta_part[seq ? 0 : part];
  if (r1 > r0) {
    // the dense sampler's apply (which every sample follows) zeroed queue[0]
    if (c->sampler != LDA_SAMPLER_DENSE || part > 0)
      HIP_TRY(hipMemsetAsync(c->queue + part, 0, sizeof(int32_t), c->stream));
    lda::SampleParams p = c->params(false);
    p.range_doc = (seq ? sch.range_doc : c->range_doc) + r0;
    p.range_end = (seq ? sch.range_end : c->range_doc + 1) + r0;
    p.num_ranges = r1 - r0;
    p.queue = c->queue + part;
    p.delta = c->sweep_recount ? nullptr : buf;   // recount: the sampler writes z only
    p.zw = c->sweep_zw ? c->zw : nullptr;
    p.zpos = c->sweep_zw ? c->zpos : nullptr;
    // (the sparse apply recomputes the nwsum delta from the nw delta
    // (k_apply_cols) and drops what a sampler put there)
    p.dsum = c->sweep_recount ? nullptr : buf + (int64_t)c->V * c->Kp;
    const int64_t wpb = c->waves_per_block;
    // a split sweep leaves reserve_cus CUs' worth of sampler blocks free, so
    // the collective of the part before this one finds CUs to run on
    int64_t cap = c->sample_blocks;
    if (c->parts > 1 && !seq && c->reserve_cus > 0)
      cap = std::max<int64_t>(1, (int64_t)c->sample_blocks * std::max(1, c->cus - c->reserve_cus) / c->cus);
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(cap, (r1 - r0 + wpb - 1) / wpb));
    const int slot = (int)(c->launches % lda_ctx::LDA_TIME_RING);
    HIP_TRY(hipEventRecord(c->ev0[slot], c->stream));
    // a probe sweep times its first launch (part 0 unless that part is empty)
    const int probe = c->big_probe_slot >= 0 && c->big_ev_tag[c->big_probe_slot] < 0 ? c->big_probe_slot : -1;
    if (probe >= 0) {
      c->big_ev_tag[probe] = ((int64_t)(r1 - r0) << 16) | ((int64_t)c->sweep_kind << 8) | part;
      HIP_TRY(hipEventRecord(c->big_ev[probe][0], c->stream));
    }
#ifdef SB_X_DELTA_KERNEL
    // measurement builds only (tools/build_variant.sh): the large-K sampler
    // without its delta atomics, the changes made by k_delta_from_z from a
    // copy of z taken before the pass (plain one-part sweeps of the whole shard)
    static int32_t* zold = nullptr;
    static int64_t zold_n = 0;
    const bool dz = c->sampler == LDA_SAMPLER_SPARSE && c->C >= 32 && !seq && c->parts == 1 && !c->sweep_recount;
    if (dz) {
      if (zold_n < c->N) {
        if (zold) HIP_TRY(hipFree(zold));
        HIP_TRY(hipMalloc(&zold, sizeof(int32_t) * (size_t)c->N));
        zold_n = c->N;
      }
      HIP_TRY(hipMemcpyAsync(zold, c->z, sizeof(int32_t) * (size_t)c->N, hipMemcpyDeviceToDevice, c->stream));
    } else if (c->sampler == LDA_SAMPLER_SPARSE && c->C >= 32) {
      return fail(LDA_ERR_UNSUPPORTED, "SB_X_DELTA_KERNEL build: plain one-part sweeps only");
    }
#endif
    if (c->sampler == LDA_SAMPLER_SPARSE)
      HIP_TRY(lda::launch_sample_sparse(c->C, false, p, blocks, c->stream, c->big_rb));
    else
      HIP_TRY(lda::launch_sample(c->C, false, p, blocks, c->stream, c->half));
    if (probe >= 0) HIP_TRY(hipEventRecord(c->big_ev[probe][1], c->stream));
    HIP_TRY(hipEventRecord(c->ev1[slot], c->stream));
#ifdef SB_X_DELTA_KERNEL
    if (dz) HIP_TRY(lda::launch_delta_from_z(c->words, zold, c->z, c->N, c->Kp, buf, c->stream));
#endif
    if (c->sweep_recount) {
      // a split sweep: this part's rows recounted into its exchange buffer
      // (the apply left it zero; the parts' buffers sum to the counts); a
      // sequential sweep: every token (the parts sampled so far with their
      // new topics, the rest with their old ones) into buffer 0, whose
      // counts the apply between the parts sets
      const int64_t i0 = seq ? 0 : c->part_item[(size_t)part];
      const int64_t i1 = seq ? c->part_item[(size_t)c->parts] : c->part_item[(size_t)part + 1];
      HIP_TRY(lda::launch_recount(c->Kp, c->perm, c->sweep_zw ? c->zw : nullptr, c->items + 4 * i0,
                                  (int32_t)(i1 - i0), c->z, buf, buf + (int64_t)c->V * c->Kp,
                                  c->recount_blocks, c->stream));
    }
    HIP_TRY(hipEventRecord(c->ev2[slot], c->stream));
    c->recounted[slot] = c->sweep_recount;
    c->launches++;
  } else if (c->sweep_recount && seq && c->N > 0) {
    // a sequential part with no documents here: the shard's counts are still
    // the ones the apply between the parts sets
    HIP_TRY(lda::launch_recount(c->Kp, c->perm, c->sweep_zw ? c->zw : nullptr, c->items,
                                (int32_t)c->part_item[(size_t)c->parts], c->z, buf, buf + (int64_t)c->V * c->Kp,
                                c->recount_blocks, c->stream));
  }
  c->pending = true;  // the part buffers hold this sweep's changes
  c->pending_absolute = c->sweep_recount;
  if (++c->next_part == nparts) {
    c->next_part = 0;
    c->sweep++;
    c->sweeps_since_seed++;
  }
  return LDA_OK;
}

lda_status lda_sample(lda_ctx* c) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (c->next_part != 0) return fail(LDA_ERR_STATE, "lda_sample inside a split sweep: finish it with lda_sample_part");
  // a warm-start sweep applies each part before the next one samples; its
  // last part stays pending for the caller's lda_apply, like any sweep
  const int n = sweep_parts(c);
  for (int i = 0; i < n; ++i) {
    lda_status s = sample_part_impl(c, i);
    if (s == LDA_OK && c->sweep_seq && i + 1 < n) s = apply_impl(c);
    if (s) return s;
  }
  return LDA_OK;
  });
}

lda_status lda_sample_part(lda_ctx* c, int32_t part) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (part < 0 || part >= sweep_parts(c)) return fail(LDA_ERR_INVALID_ARG, "part out of range [0, parts)");
  return sample_part_impl(c, part);
  });
}

lda_status lda_set_exchange_parts(lda_ctx* c, int32_t parts, int32_t reserve_cus) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (parts < 1 || parts > LDA_MAX_EXCHANGE_PARTS)
    return fail(LDA_ERR_INVALID_ARG, "parts must be in [1, LDA_MAX_EXCHANGE_PARTS]");
  // < 0: the default, 1/32 of the CUs (8 on MI355X's 256; C4 split-sweep A/B
  // on one GPU: DESIGN.md §5)
  if (reserve_cus < 0) reserve_cus = std::max(1, c->cus / 32);
  if (c->next_part != 0) return fail(LDA_ERR_STATE, "inside a split sweep");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipStreamSynchronize(c->stream));
  const size_t cells = (size_t)c->V * c->Kp + c->Kp;
  for (int i = 1; i < LDA_MAX_EXCHANGE_PARTS; ++i) {
    if (i < parts && !c->delta_part[i]) {
      HIP_TRY(dalloc(&c->delta_part[i], cells));
      HIP_TRY(hipMemsetAsync(c->delta_part[i], 0, sizeof(int32_t) * cells, c->stream));
    } else if (i >= parts && c->delta_part[i]) {
      // a pending change in a dropped part goes to part 0 first
      HIP_TRY(lda::launch_fold_delta(c->delta, c->delta_part[i], (int64_t)cells, c->stream));
      HIP_TRY(hipStreamSynchronize(c->stream));
      HIP_TRY(hipFree(c->delta_part[i]));
      c->delta_part[i] = nullptr;
    }
  }
  std::vector<int64_t> pr;
  std::vector<int64_t> ranges = make_part_ranges(c->doc_off_h, c->tokens_per_range, parts, pr);
  int64_t* dr = nullptr;
  HIP_TRY(dalloc(&dr, ranges.size()));
  hipError_t e = hipMemcpyAsync(dr, ranges.data(), sizeof(int64_t) * ranges.size(), hipMemcpyHostToDevice, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) (void)hipFree(dr);
  HIP_TRY(e);
  (void)hipFree(c->range_doc);
  c->range_doc = dr;
  c->graph_key = lda_ctx::GraphKey{};   // the graphs captured the old ranges
  c->R = (int64_t)ranges.size() - 1;
  c->part_range = pr;
  c->ranges_h = ranges;
  c->parts = parts;
  c->reserve_cus = reserve_cus;
  return c->perm ? build_recount_index(c) : LDA_OK;   // the index is per part
  });
}

lda_status lda_get_exchange_parts(lda_ctx* c, int32_t* parts) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !parts) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *parts = c->parts;
  return LDA_OK;
  });
}

lda_status lda_delta_buffer_part(lda_ctx* c, int32_t part, void** dev_ptr, size_t* count) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !dev_ptr || !count) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (part < 0 || part >= sweep_parts(c)) return fail(LDA_ERR_INVALID_ARG, "part out of range [0, parts)");
  // a warm-start sweep's parts all go through buffer 0
  const bool seq = c->next_part != 0 || c->pending ? c->sweep_seq : next_sweep_sequential(c);
  *dev_ptr = c->delta_part[seq ? 0 : part];
  *count = (size_t)c->V * c->Kp + c->Kp;
  return LDA_OK;
  });
}

// ---- compact exchange
static lda_status exchange_dims(lda_ctx* c, int32_t world, int64_t max_tokens, size_t* packed_count,
                                size_t* escape_count, int32_t* cap) {
  // world 1: the sum is the identity (a one-rank run with the exchange forced on, to exercise it)
  const int per = c->exch_cells;
  const int max_world = per == 4 ? 64 : 16384;
  if (world < 1 || world > max_world)
    return fail(LDA_ERR_INVALID_ARG, per == 4 ? "world must be in [1, 64] with 4 cells per word"
                                              : "world must be in [1, 16384]");
  if (max_tokens < c->N) return fail(LDA_ERR_INVALID_ARG, "max_shard_tokens below this shard's tokens");
  // sum |cell| of one rank's buffer <= 2 x its tokens, so at most that over
  // the smallest bias can escape
  const int64_t bmin = per == 4 ? lda::exch_bias4_top(world) : lda::exch_bias1(world);
  const int64_t k = 2 * max_tokens / bmin + 1;
  if (k > (int64_t)INT32_MAX / 3 - 1) return fail(LDA_ERR_UNSUPPORTED, "escape list beyond int32 indexing");
  *cap = (int32_t)k;
  *packed_count = (size_t)c->V * c->Kp / per + c->Kp;
  *escape_count = 1 + 3 * (size_t)k;
  return LDA_OK;
}

// the buffer slot a part's changes are in (a warm-start sweep: always 0)
static int exchange_slot(lda_ctx* c, int32_t part) {
  const bool seq = c->next_part != 0 || c->pending ? c->sweep_seq : next_sweep_sequential(c);
  return seq ? 0 : part;
}

lda_status lda_set_exchange_cells(lda_ctx* c, int32_t cells_per_word) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (cells_per_word != 2 && cells_per_word != 4) return fail(LDA_ERR_INVALID_ARG, "cells_per_word must be 2 or 4");
  if (c->exch_cells != cells_per_word) {
    // the packed words of a pending exchange have the old layout
    for (int i = 0; i < LDA_MAX_EXCHANGE_PARTS; ++i)
      if (c->exch_packed[i]) {
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipFree(c->exch_packed[i]));
        c->exch_packed[i] = nullptr;
      }
    c->exch_cells = cells_per_word;
  }
  return LDA_OK;
  });
}

lda_status lda_get_exchange_cells(lda_ctx* c, int32_t* cells_per_word) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !cells_per_word) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *cells_per_word = c->exch_cells;
  return LDA_OK;
  });
}

lda_status lda_exchange_sizes(lda_ctx* c, int32_t world, int64_t max_shard_tokens, size_t* packed_count,
                              size_t* escape_count) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !packed_count || !escape_count) return fail(LDA_ERR_INVALID_ARG, "null argument");
  int32_t cap = 0;
  return exchange_dims(c, world, max_shard_tokens, packed_count, escape_count, &cap);
  });
}

lda_status lda_exchange_pack(lda_ctx* c, int32_t part, int32_t world, int64_t max_shard_tokens, void** packed,
                             void** escapes) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !packed || !escapes) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (part < 0 || part >= sweep_parts(c)) return fail(LDA_ERR_INVALID_ARG, "part out of range [0, parts)");
  size_t np = 0, ne = 0;
  int32_t cap = 0;
  lda_status s = exchange_dims(c, world, max_shard_tokens, &np, &ne, &cap);
  if (s) return s;
  const int slot = exchange_slot(c, part);
  HIP_TRY(hipSetDevice(c->device));
  if (!c->exch_packed[slot]) HIP_TRY(dalloc(&c->exch_packed[slot], np));
  if (c->exch_esc_cap[slot] < ne) {
    if (c->exch_esc[slot]) HIP_TRY(hipFree(c->exch_esc[slot]));
    c->exch_esc[slot] = nullptr;
    c->exch_esc_cap[slot] = 0;
    HIP_TRY(dalloc(&c->exch_esc[slot], ne));
    c->exch_esc_cap[slot] = ne;
  }
  const int64_t cells = (int64_t)c->V * c->Kp;
  int32_t* buf = c->delta_part[slot];
  int32_t* pk = c->exch_packed[slot];
  int32_t* es = c->exch_esc[slot];
  HIP_TRY(hipMemsetAsync(es, 0, sizeof(int32_t), c->stream));
  HIP_TRY(lda::launch_exch_pack(buf, cells, pk, world, es, cap, c->stream, c->exch_cells));
  HIP_TRY(hipMemcpyAsync(pk + cells / c->exch_cells, buf + cells, sizeof(int32_t) * c->Kp,
                         hipMemcpyDeviceToDevice, c->stream));
  *packed = pk;
  *escapes = es;
  return LDA_OK;
  });
}

lda_status lda_exchange_unpack(lda_ctx* c, int32_t part, int32_t world, int64_t max_shard_tokens,
                               const void* escapes_all) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !escapes_all) return fail(LDA_ERR_INVALID_ARG, "null argument");
  size_t np = 0, ne = 0;
  int32_t cap = 0;
  lda_status s = exchange_dims(c, world, max_shard_tokens, &np, &ne, &cap);
  if (s) return s;
  return lda_exchange_unpack_lists(c, part, world, max_shard_tokens, escapes_all, cap);
  });
}

lda_status lda_exchange_unpack_lists(lda_ctx* c, int32_t part, int32_t world, int64_t max_shard_tokens,
                                     const void* escapes_all, int32_t list_cap) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (part < 0 || part >= sweep_parts(c)) return fail(LDA_ERR_INVALID_ARG, "part out of range [0, parts)");
  size_t np = 0, ne = 0;
  int32_t cap = 0;
  lda_status s = exchange_dims(c, world, max_shard_tokens, &np, &ne, &cap);
  if (s) return s;
  if (list_cap < 0 || list_cap > cap) return fail(LDA_ERR_INVALID_ARG, "list_cap out of range [0, escape capacity]");
  if (!escapes_all && list_cap > 0) return fail(LDA_ERR_INVALID_ARG, "null escapes_all with list_cap > 0");
  cap = list_cap;
  const int slot = exchange_slot(c, part);
  if (!c->exch_packed[slot]) return fail(LDA_ERR_STATE, "lda_exchange_unpack before lda_exchange_pack");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t cells = (int64_t)c->V * c->Kp;
  int32_t* buf = c->delta_part[slot];
  const int32_t* pk = c->exch_packed[slot];
  HIP_TRY(hipMemcpyAsync(buf + cells, pk + cells / c->exch_cells, sizeof(int32_t) * c->Kp,
                         hipMemcpyDeviceToDevice, c->stream));
  HIP_TRY(lda::launch_exch_unpack(pk, cells, buf, world,
                                  list_cap > 0 ? static_cast<const int32_t*>(escapes_all) : nullptr, cap,
                                  c->stream, c->exch_cells));
  return LDA_OK;
  });
}

lda_status lda_counts_checksum(lda_ctx* c, uint64_t* checksum) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !checksum) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (c->pending) return fail(LDA_ERR_STATE, "checksum with a pending delta: call lda_apply first");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t n4 = (int64_t)c->V * c->Kp / 4;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 2048));
  uint64_t* part = nullptr;
  HIP_TRY(dalloc(&part, (size_t)blocks));
  std::vector<uint64_t> h((size_t)blocks);
  hipError_t e = lda::launch_counts_checksum(c->nw, c->nwsum, c->K, c->Kp, c->V, part, blocks, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), part, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(part);
  HIP_TRY(e);
  uint64_t s = 0;
  for (uint64_t x : h) s += x;
  *checksum = s;
  return LDA_OK;
  });
}

// Debug (not in the public header): one sparse sampling pass that also
// records 8 floats per token (kn, sumB, sumA, thr, nnz, z_old, word, u).
lda_status lda_debug_sample_trace(lda_ctx* c, float* host_trace) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !host_trace) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (c->pending) return fail(LDA_ERR_STATE, "pending delta");
  if (c->sampler != LDA_SAMPLER_SPARSE) return fail(LDA_ERR_UNSUPPORTED, "sparse sampler only");
  HIP_TRY(hipSetDevice(c->device));
  float* tr = nullptr;
  HIP_TRY(dalloc(&tr, (size_t)8 * std::max<int64_t>(c->N, 1)));
  // zeroed: measurement builds of the large-K sampler count into it
  hipError_t e = hipMemsetAsync(tr, 0, sizeof(float) * 8 * std::max<int64_t>(c->N, 1), c->stream);
  if (e == hipSuccess) e = hipMemsetAsync(c->queue, 0, sizeof(int32_t), c->stream);
  lda::SampleParams p = c->params(false);
  p.trace = tr;
  const int64_t wpb = c->waves_per_block;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(c->sample_blocks, (c->R + wpb - 1) / wpb));
  if (e == hipSuccess && c->N > 0) e = lda::launch_sample_sparse(c->C, false, p, blocks, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(host_trace, tr, sizeof(float) * 8 * c->N, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(tr);
  HIP_TRY(e);
  c->sweep++;
  c->pending = true;
  return LDA_OK;
  });
}

lda_status lda_last_sample_ms(lda_ctx* c, float* ms) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !ms) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *ms = 0.0f;
  if (c->launches == 0) return LDA_OK;
  const int slot = (int)((c->launches - 1) % lda_ctx::LDA_TIME_RING);
  HIP_TRY(hipEventSynchronize(c->ev1[slot]));
  HIP_TRY(hipEventElapsedTime(ms, c->ev0[slot], c->ev1[slot]));
  return LDA_OK;
  });
}

lda_status lda_philox_draws(uint64_t seed, uint32_t c2, uint32_t c3, const int64_t* gtok, int64_t n,
                            uint32_t* out) {
  return lda_abi::guarded([&]() -> lda_status {
  if (n < 0 || (n > 0 && (!gtok || !out))) return fail(LDA_ERR_INVALID_ARG, "bad argument");
  if (n == 0) return LDA_OK;
  int64_t* dg = nullptr;
  uint32_t* dout = nullptr;
  hipError_t e = hipMalloc(&dg, sizeof(int64_t) * n);
  if (e == hipSuccess) e = hipMalloc(&dout, sizeof(uint32_t) * n);
  if (e == hipSuccess) e = hipMemcpy(dg, gtok, sizeof(int64_t) * n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = lda::launch_philox_draws(dg, n, c2, c3, seed, dout, nullptr);
  if (e == hipSuccess) e = hipMemcpy(out, dout, sizeof(uint32_t) * n, hipMemcpyDeviceToHost);
  (void)hipFree(dg);
  (void)hipFree(dout);
  HIP_TRY(e);
  return LDA_OK;
  });
}

lda_status lda_sample_times(lda_ctx* c, int32_t max, float* ms, int32_t* n) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !n || max < 0 || (max > 0 && !ms)) return fail(LDA_ERR_INVALID_ARG, "bad argument");
  const int64_t avail = std::min<int64_t>(c->launches, lda_ctx::LDA_TIME_RING);
  const int32_t k = (int32_t)std::min<int64_t>(avail, max);
  *n = k;
  for (int32_t i = 0; i < k; ++i) {
    const int slot = (int)((c->launches - k + i) % lda_ctx::LDA_TIME_RING);
    HIP_TRY(hipEventSynchronize(c->ev1[slot]));
    HIP_TRY(hipEventElapsedTime(&ms[i], c->ev0[slot], c->ev1[slot]));
  }
  return LDA_OK;
  });
}

lda_status lda_recount_times(lda_ctx* c, int32_t max, float* ms, int32_t* n) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !n || max < 0 || (max > 0 && !ms)) return fail(LDA_ERR_INVALID_ARG, "bad argument");
  const int64_t avail = std::min<int64_t>(c->launches, lda_ctx::LDA_TIME_RING);
  const int32_t k = (int32_t)std::min<int64_t>(avail, max);
  *n = k;
  for (int32_t i = 0; i < k; ++i) {
    const int slot = (int)((c->launches - k + i) % lda_ctx::LDA_TIME_RING);
    ms[i] = 0.0f;                      // a delta-mode launch runs no recount
    if (!c->recounted[slot]) continue;
    HIP_TRY(hipEventSynchronize(c->ev2[slot]));
    HIP_TRY(hipEventElapsedTime(&ms[i], c->ev1[slot], c->ev2[slot]));
  }
  return LDA_OK;
  });
}

// (re)builds a sequential schedule's work ranges on the device
static lda_status build_schedule(lda_ctx* c, const std::vector<int64_t>& cum, int64_t g0, int64_t gn,
                                 lda_ctx::SeqSchedule& sch) {
  const int parts = (int)cum.size() - 1;
  if (parts > 1) {
    std::vector<int64_t> pr, st, en;
    make_run_ranges(c->doc_off_h, c->tokens_per_range, seq_part_runs(c->doc_off_h, cum, c->token_base, g0, gn),
                    st, en, pr);
    // one device buffer: starts [R] then ends [R]
    const size_t R = st.size();
    st.insert(st.end(), en.begin(), en.end());
    int64_t* dr = nullptr;
    HIP_TRY(dalloc(&dr, st.size()));
    hipError_t e = hipMemcpyAsync(dr, st.data(), sizeof(int64_t) * st.size(), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) (void)hipFree(dr);
    HIP_TRY(e);
    if (sch.range_doc) (void)hipFree(sch.range_doc);
    sch.range_doc = dr;
    sch.range_end = dr + R;
    sch.part_range = pr;
  }
  sch.parts = parts;
  sch.cum = cum;
  return LDA_OK;
}

lda_status lda_set_warm_start(lda_ctx* c, int32_t parts, int32_t sweeps, int64_t corpus_first_token,
                              int64_t corpus_tokens) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (parts < 1 || parts > LDA_MAX_EXCHANGE_PARTS || sweeps < 0)
    return fail(LDA_ERR_INVALID_ARG, "parts must be in [1, LDA_MAX_EXCHANGE_PARTS], sweeps >= 0");
  if (c->next_part != 0) return fail(LDA_ERR_STATE, "inside a split sweep");
  if (corpus_tokens <= 0) {          // this shard is the whole corpus
    corpus_first_token = c->token_base;
    corpus_tokens = c->N;
  }
  HIP_TRY(hipSetDevice(c->device));
  lda_status s = build_schedule(c, equal_cum(parts), corpus_first_token, corpus_tokens, c->warm);
  if (s) return s;
  c->warm_sweeps = parts > 1 ? sweeps : 0;
  c->graph_key = lda_ctx::GraphKey{};
  return LDA_OK;
  });
}

// fractions[parts] > 0 summing to 1 -> cumulative units of 1 / LDA_SEQ_FRACTION_UNIT
static bool quantise_fractions(int32_t parts, const double* fractions, std::vector<int64_t>& cum) {
  cum.assign((size_t)parts + 1, 0);
  double acc = 0.0;
  for (int i = 0; i < parts; ++i) {
    if (!(fractions[i] > 0.0)) return false;
    acc += fractions[i];
    cum[(size_t)i + 1] = i + 1 == parts ? LDA_SEQ_FRACTION_UNIT
                                        : (int64_t)std::llround(acc * (double)LDA_SEQ_FRACTION_UNIT);
    if (cum[(size_t)i + 1] <= cum[(size_t)i]) return false;
  }
  return std::fabs(acc - 1.0) <= 1e-9 && cum[(size_t)parts - 1] < LDA_SEQ_FRACTION_UNIT;
}

lda_status lda_set_sequential_sweeps(lda_ctx* c, int32_t parts, const double* fractions, int64_t corpus_first_token,
                                     int64_t corpus_tokens) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (parts < 1 || parts > LDA_MAX_EXCHANGE_PARTS)
    return fail(LDA_ERR_INVALID_ARG, "parts must be in [1, LDA_MAX_EXCHANGE_PARTS]");
  std::vector<int64_t> cum;
  if (parts > 1 && !fractions) cum = equal_cum(parts);
  else if (parts > 1 && !quantise_fractions(parts, fractions, cum))
    return fail(LDA_ERR_INVALID_ARG, "fractions must be > 0, increasing when quantised, and sum to 1");
  if (parts == 1) cum = equal_cum(1);
  if (c->next_part != 0) return fail(LDA_ERR_STATE, "inside a split sweep");
  if (corpus_tokens <= 0) {
    corpus_first_token = c->token_base;
    corpus_tokens = c->N;
  }
  HIP_TRY(hipSetDevice(c->device));
  lda_status s = build_schedule(c, cum, corpus_first_token, corpus_tokens, c->steady);
  if (s) return s;
  c->graph_key = lda_ctx::GraphKey{};
  return LDA_OK;
  });
}

lda_status lda_get_sequential_sweeps(lda_ctx* c, int32_t* parts, int64_t* cum_units) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (parts) *parts = c->steady.parts;
  if (cum_units)
    for (size_t i = 0; i < c->steady.cum.size(); ++i) cum_units[i] = c->steady.cum[i];
  return LDA_OK;
  });
}

lda_status lda_staleness_schedule(int32_t threads, int32_t* parts, double* fractions) {
  return lda_abi::guarded([&]() -> lda_status {
  if (threads < 1 || !parts || !fractions) return fail(LDA_ERR_INVALID_ARG, "threads >= 1 and outputs needed");
  if (threads == 1) {
    // sequential Mallet (mean live fraction 1/2): the most parts allowed
    *parts = LDA_MAX_EXCHANGE_PARTS;
    for (int i = 0; i < *parts; ++i) fractions[i] = 1.0 / *parts;
    return LDA_OK;
  }
  // two parts, the first a fraction f of every block: its tokens see none of
  // the sweep's changes, the second part's see f, so the mean live fraction
  // is f (1 - f) = 1 / (2 T), Mallet's with T worker threads
  const double f = 0.5 * (1.0 - std::sqrt(1.0 - 2.0 / threads));
  *parts = 2;
  fractions[0] = f;
  fractions[1] = 1.0 - f;
  return LDA_OK;
  });
}

lda_status lda_warm_part_tokens(const int64_t* doc_off, int64_t num_docs, int32_t parts, int64_t token_base,
                                int64_t corpus_first_token, int64_t corpus_tokens, int64_t* tokens_out) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!doc_off || !tokens_out || num_docs < 0 || parts < 1 || parts > LDA_MAX_EXCHANGE_PARTS || corpus_tokens <= 0)
    return fail(LDA_ERR_INVALID_ARG, "null pointer, num_docs < 0, parts outside [1, LDA_MAX_EXCHANGE_PARTS] or corpus_tokens <= 0");
  std::vector<int64_t> off(doc_off, doc_off + num_docs + 1);
  for (auto& o : off) o -= doc_off[0];
  const auto runs = seq_part_runs(off, equal_cum(parts), token_base, corpus_first_token, corpus_tokens);
  for (int i = 0; i < parts; ++i) {
    int64_t n = 0;
    for (const auto& r : runs[(size_t)i]) n += off[(size_t)r.second] - off[(size_t)r.first];
    tokens_out[i] = n;
  }
  return LDA_OK;
  });
}

lda_status lda_get_warm_start(lda_ctx* c, int32_t* parts, int32_t* sweeps) {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (parts) *parts = c->warm.parts;
  if (sweeps) *sweeps = c->warm_sweeps;
  return LDA_OK;
}

lda_status lda_sweep_parts(lda_ctx* c, int32_t* parts, int32_t* sequential) {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  const bool seq = c->next_part != 0 ? c->sweep_seq : next_sweep_sequential(c);
  if (parts) *parts = seq ? seq_schedule(c).parts : c->parts;
  if (sequential) *sequential = seq ? 1 : 0;
  return LDA_OK;
}

lda_status lda_set_count_update(lda_ctx* c, int32_t mode, int32_t recount_sweeps) {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (mode != LDA_COUNT_AUTO && mode != LDA_COUNT_RECOUNT && mode != LDA_COUNT_DELTA)
    return fail(LDA_ERR_INVALID_ARG, "mode must be LDA_COUNT_AUTO, _RECOUNT or _DELTA");
  if (c->next_part != 0) return fail(LDA_ERR_STATE, "inside a split sweep");
  if (mode == LDA_COUNT_RECOUNT && !c->recount_ok)
    return fail(LDA_ERR_UNSUPPORTED, "the recount needs the dense sampler and < 2^32 tokens");
  c->count_mode = mode;
  if (mode == LDA_COUNT_AUTO && recount_sweeps >= 0) c->recount_sweeps = c->recount_ok ? recount_sweeps : 0;
  return LDA_OK;
}

lda_status lda_get_count_update(lda_ctx* c, int32_t* mode, int32_t* recount_sweeps) {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (mode) *mode = c->count_mode;
  if (recount_sweeps) *recount_sweeps = c->recount_sweeps;
  return LDA_OK;
}

lda_status lda_count_update_mode(lda_ctx* c, int32_t* recount) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !recount) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *recount = (c->pending ? c->pending_absolute : next_sweep_recounts(c)) ? 1 : 0;
  return LDA_OK;
  });
}

lda_status lda_delta_buffer(lda_ctx* c, void** dev_ptr, size_t* count) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !dev_ptr || !count) return fail(LDA_ERR_INVALID_ARG, "null argument");
  *dev_ptr = c->delta;
  *count = (size_t)c->V * c->Kp + c->Kp;
  return LDA_OK;
  });
}

// Can the next sweep run inside a graph?  A plain dense sweep: one part, not
// a warm-start or recount sweep (and once one is, every later one is).
// Steady sequential sweeps (lda_set_sequential_sweeps) qualify too: their
// parts go into the graph one after the other, each followed by its apply.
static bool graph_eligible(const lda_ctx* c) {
  return c->use_graphs && c->sampler == LDA_SAMPLER_DENSE && c->parts == 1 && c->R > 0 && !c->pending &&
         c->next_part == 0 && next_sweep_kind(c) != 1 && !next_sweep_recounts(c);
}

// k sweeps captured on the context's stream and instantiated once: k x
// (sampler, apply), or for steady sequential sweeps k x parts x (sampler
// over the part's ranges, apply), where only a sweep's last apply advances
// the device sweep counter and every part takes work-queue counter 0 (the
// apply before it zeroed it)
static lda_status sweep_graph(lda_ctx* c, int k, hipGraphExec_t* out) {
  const bool seq = next_sweep_kind(c) == 2;
  lda_ctx::GraphKey key;
  key.range_doc = c->range_doc;
  key.R = c->R;
  key.stream = c->stream;
  key.seq = seq ? c->steady.range_doc : nullptr;
  key.seq_parts = seq ? c->steady.parts : 0;
  if (!(key == c->graph_key)) {
    // a graph launched earlier (perhaps on another stream: lda_set_stream does
    // not synchronize) may still run; it finishes before it is destroyed
    if (c->graph_ev_live) HIP_TRY(hipEventSynchronize(c->graph_ev));
    c->graph_ev_live = false;
    for (auto& g : c->graphs)
      if (g) {
        (void)hipGraphExecDestroy(g);
        g = nullptr;
      }
    c->graph_key = key;
  }
  if (!c->graphs[k]) {
    lda::SampleParams p = c->params(false);
    p.state_dev = c->state_dev;
    p.delta = c->delta;
    p.dsum = c->delta + (int64_t)c->V * c->Kp;
    const int64_t wpb = c->waves_per_block;
    auto blocks_for = [&](int64_t R) {
      return (int)std::max<int64_t>(1, std::min<int64_t>(c->sample_blocks, (R + wpb - 1) / wpb));
    };
    lda::TopicTables t{c->nwsum, c->alpha_d, c->alpha_f, c->inv, c->inv_m1, 0.0f, c->K, c->queue, 0,
                       c->state_dev, 1};
    lda::TopicTables t_part = t;
    t_part.advance = 0;
    HIP_TRY(hipStreamBeginCapture(c->stream, hipStreamCaptureModeRelaxed));
    hipError_t e = hipSuccess;
    for (int i = 0; i < k && e == hipSuccess; ++i) {
      if (!seq) {
        e = lda::launch_sample(c->C, false, p, blocks_for(c->R), c->stream, c->half);
        if (e == hipSuccess) e = lda::launch_apply_packed(c->nw, c->delta, c->V, c->Kp, c->nw16, c->wide, t, c->stream);
        continue;
      }
      for (int part = 0; part < c->steady.parts && e == hipSuccess; ++part) {
        const int64_t r0 = c->steady.part_range[(size_t)part], r1 = c->steady.part_range[(size_t)part + 1];
        lda::SampleParams pp = p;
        pp.range_doc = c->steady.range_doc + r0;
        pp.range_end = c->steady.range_end + r0;
        pp.num_ranges = r1 - r0;
        if (r1 > r0) e = lda::launch_sample(c->C, false, pp, blocks_for(r1 - r0), c->stream, c->half);
        const bool last = part + 1 == c->steady.parts;
        if (e == hipSuccess)
          e = lda::launch_apply_packed(c->nw, c->delta, c->V, c->Kp, c->nw16, c->wide, last ? t : t_part,
                                       c->stream);
      }
    }
    hipGraph_t g = nullptr;
    const hipError_t e2 = hipStreamEndCapture(c->stream, &g);
    if (e == hipSuccess) e = e2;
    if (e == hipSuccess) e = hipGraphInstantiate(&c->graphs[k], g, nullptr, nullptr, 0);
    if (g) (void)hipGraphDestroy(g);
    HIP_TRY(e);
  }
  *out = c->graphs[k];
  return LDA_OK;
}

lda_status lda_sweep(lda_ctx* c, int32_t n) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (n < 0) return fail(LDA_ERR_INVALID_ARG, "n must be >= 0");
  if (c->pending) {
    lda_status s = apply_impl(c);
    if (s) return s;
  }
  for (int32_t i = 0; i < n;) {
    if (graph_eligible(c)) {
      // the rest as graphs of up to GRAPH_MAX sweeps
      const int k = (int)std::min<int32_t>(n - i, lda_ctx::GRAPH_MAX);
      hipGraphExec_t g = nullptr;
      HIP_TRY(hipSetDevice(c->device));
      lda_status s = sweep_graph(c, k, &g);
      if (s) return s;
      auto word = [&](int i) { return reinterpret_cast<hipDeviceptr_t>(c->state_dev + i); };
      if (!c->state_beta) {
        const float b = (float)c->beta, vb = (float)((double)c->V * c->beta);
        HIP_TRY(hipMemsetD32Async(word(1), (int)__builtin_bit_cast(uint32_t, b), 1, c->stream));
        HIP_TRY(hipMemsetD32Async(word(2), (int)__builtin_bit_cast(uint32_t, vb), 1, c->stream));
        c->state_beta = true;
      }
      if (c->state_sweep != (int64_t)c->sweep)
        HIP_TRY(hipMemsetD32Async(word(0), (int)c->sweep, 1, c->stream));
      HIP_TRY(hipGraphLaunch(g, c->stream));
      if (!c->graph_ev) HIP_TRY(hipEventCreateWithFlags(&c->graph_ev, hipEventDisableTiming));
      HIP_TRY(hipEventRecord(c->graph_ev, c->stream));
      c->graph_ev_live = true;
      c->state_sweep = (int64_t)c->sweep + k;
      c->sweep += (uint32_t)k;
      c->sweeps_since_seed += k;
      c->sweep_seq = false;
      c->sweep_recount = false;
      c->zw_valid = false;
      c->pending_absolute = false;
      c->apply_gen += (uint64_t)k;
      i += k;
      continue;
    }
    lda_status s = lda_sample(c);
    if (s) return s;
    s = apply_impl(c);
    if (s) return s;
    ++i;
  }
  return LDA_OK;
  });
}

lda_status lda_get_z(lda_ctx* c, int32_t* z) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !z) return fail(LDA_ERR_INVALID_ARG, "null argument");
  HIP_TRY(hipSetDevice(c->device));
  if (c->N > 0) HIP_TRY(hipMemcpyAsync(z, c->z, sizeof(int32_t) * c->N, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LDA_OK;
  });
}

lda_status lda_set_z(lda_ctx* c, const int32_t* z) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !z) return fail(LDA_ERR_INVALID_ARG, "null argument");
  for (int64_t i = 0; i < c->N; ++i)
    if (z[i] < 0 || z[i] >= c->K) return fail(LDA_ERR_INVALID_ARG, "topic out of range [0, K)");
  HIP_TRY(hipSetDevice(c->device));
  if (c->N > 0) HIP_TRY(hipMemcpyAsync(c->z, z, sizeof(int32_t) * c->N, hipMemcpyHostToDevice, c->stream));
  lda_status s = reseed_counts(c);
  if (s) return s;
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LDA_OK;
  });
}

lda_status lda_get_counts(lda_ctx* c, int32_t* nw, int32_t* nwsum, int32_t* nd, int32_t* ndsum) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  HIP_TRY(hipSetDevice(c->device));
  if (nw) {
    HIP_TRY(hipMemcpy2DAsync(nw, sizeof(int32_t) * c->K, c->nw, sizeof(int32_t) * c->Kp,
                             sizeof(int32_t) * c->K, c->V, hipMemcpyDeviceToHost, c->stream));
  }
  if (nwsum) HIP_TRY(hipMemcpyAsync(nwsum, c->nwsum, sizeof(int32_t) * c->K, hipMemcpyDeviceToHost, c->stream));
  if (nd && c->D > 0) {
    int32_t* tmp = nullptr;
    HIP_TRY(dalloc(&tmp, (size_t)c->D * c->K));
    hipError_t e = lda::launch_doc_topics(c->z, c->doc_off, c->D, c->K, c->Kp, tmp, 0, c->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(nd, tmp, sizeof(int32_t) * (size_t)c->D * c->K, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(tmp);
    HIP_TRY(e);
  }
  if (ndsum)
    for (int64_t d = 0; d < c->D; ++d) ndsum[d] = (int32_t)(c->doc_off_h[d + 1] - c->doc_off_h[d]);
  HIP_TRY(hipStreamSynchronize(c->stream));
  return LDA_OK;
  });
}

lda_status lda_set_alpha_beta(lda_ctx* c, const double* alpha, double beta) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !alpha) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (!(beta > 0.0)) return fail(LDA_ERR_INVALID_ARG, "beta must be > 0");
  for (int k = 0; k < c->K; ++k)
    if (!(alpha[k] > 0.0)) return fail(LDA_ERR_INVALID_ARG, "alpha must be > 0");
  HIP_TRY(hipSetDevice(c->device));
  if (!c->alpha_pin) {
    HIP_TRY(hipHostMalloc(&c->alpha_pin, sizeof(double) * c->K, hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&c->alpha_ev, hipEventDisableTiming));
  }
  if (c->alpha_ev_live) HIP_TRY(hipEventSynchronize(c->alpha_ev));   // the previous upload has left
  c->alpha.assign(alpha, alpha + c->K);
  c->beta = beta;
  c->state_beta = false;
  std::copy(alpha, alpha + c->K, c->alpha_pin);
  HIP_TRY(hipMemcpyAsync(c->alpha_d, c->alpha_pin, sizeof(double) * c->K, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipEventRecord(c->alpha_ev, c->stream));
  c->alpha_ev_live = true;
  // refresh the fp32 tables (the nwsum delta part is zero unless pending)
  if (!c->pending) {
    HIP_TRY(prepare_tables(c));
  }
  return LDA_OK;
  });
}

lda_status lda_log_likelihood_enqueue(lda_ctx* c, int64_t* ticket) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !ticket) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (c->pending) return fail(LDA_ERR_STATE, "log likelihood with a pending delta: call lda_apply first");
  HIP_TRY(hipSetDevice(c->device));
  const int nb = c->partial_blocks;
  lda_ctx::LLSlot& sl = c->ll[c->ll_next % lda_ctx::LL_SLOTS];
  if (!sl.host) {
    HIP_TRY(hipHostMalloc(&sl.host, sizeof(double) * 2 * nb + sizeof(unsigned long long) * nb +
                                        sizeof(int32_t) * c->K, hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  } else {
    HIP_TRY(hipEventSynchronize(sl.done));   // an uncollected older result is overwritten
  }
  double* hd = static_cast<double*>(sl.host);
  double* hw = hd + nb;
  auto* hz = reinterpret_cast<unsigned long long*>(hw + nb);
  auto* hs = reinterpret_cast<int32_t*>(hz + nb);
  double alpha_sum = 0.0;
  for (double a : c->alpha) alpha_sum += a;
  if (c->D > 0) {
    HIP_TRY(lda::launch_ll_docs(c->z, c->doc_off, c->D, c->alpha_d, alpha_sum, c->K, c->Kp,
                                c->partial, nb, c->stream));
    HIP_TRY(hipMemcpyAsync(hd, c->partial, sizeof(double) * nb, hipMemcpyDeviceToHost, c->stream));
  } else {
    std::fill(hd, hd + nb, 0.0);
  }
  // stream order: the copy above has read c->partial before k_ll_words writes it
  HIP_TRY(lda::launch_ll_words(c->nw, c->V, c->K, c->Kp, c->beta, c->partial, c->nonzero, nb, c->stream));
  HIP_TRY(hipMemcpyAsync(hw, c->partial, sizeof(double) * nb, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(hz, c->nonzero, sizeof(unsigned long long) * nb, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(hs, c->nwsum, sizeof(int32_t) * c->K, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipEventRecord(sl.done, c->stream));
  sl.alpha_sum = alpha_sum;
  sl.beta = c->beta;
  sl.ticket = c->ll_next;
  *ticket = c->ll_next++;
  return LDA_OK;
  });
}

lda_status lda_log_likelihood_collect(lda_ctx* c, int64_t ticket, double* doc_part, double* word_part) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || ticket < 0) return fail(LDA_ERR_INVALID_ARG, "bad argument");
  lda_ctx::LLSlot& sl = c->ll[ticket % lda_ctx::LL_SLOTS];
  if (sl.ticket != ticket)
    return fail(LDA_ERR_STATE, "log-likelihood ticket already collected or overwritten (at most 16 in flight)");
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipEventSynchronize(sl.done));
  const int nb = c->partial_blocks;
  const double* hd = static_cast<const double*>(sl.host);
  const double* hw = hd + nb;
  const auto* hz = reinterpret_cast<const unsigned long long*>(hw + nb);
  const auto* hs = reinterpret_cast<const int32_t*>(hz + nb);
  double docs = 0.0, words_ll = 0.0;
  unsigned long long nonzero = 0;
  for (int b = 0; b < nb; ++b) {
    docs += hd[b];
    words_ll += hw[b];
    nonzero += hz[b];
  }
  docs += (double)c->D * log_gamma_stirling(sl.alpha_sum);
  for (int k = 0; k < c->K; ++k) words_ll -= log_gamma_stirling(sl.beta * c->V + hs[k]);
  words_ll += log_gamma_stirling(sl.beta * c->V) * c->K;
  words_ll -= log_gamma_stirling(sl.beta) * (double)nonzero;
  if (doc_part) *doc_part = docs;
  if (word_part) *word_part = words_ll;
  sl.ticket = -1;
  return LDA_OK;
  });
}

lda_status lda_log_likelihood_parts(lda_ctx* c, double* doc_part, double* word_part) {
  return lda_abi::guarded([&]() -> lda_status {
  int64_t t = -1;
  lda_status s = lda_log_likelihood_enqueue(c, &t);
  if (s) return s;
  return lda_log_likelihood_collect(c, t, doc_part, word_part);
  });
}

lda_status lda_log_likelihood(lda_ctx* c, double* out) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!out) return fail(LDA_ERR_INVALID_ARG, "null argument");
  double a = 0.0, b = 0.0;
  lda_status s = lda_log_likelihood_parts(c, &a, &b);
  if (s) return s;
  *out = a + b;
  return LDA_OK;
  });
}

lda_status lda_max_doc_length(lda_ctx* c, int32_t* max_len) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !max_len) return fail(LDA_ERR_INVALID_ARG, "null argument");
  int64_t m = 0;
  for (int64_t d = 0; d < c->D; ++d) m = std::max(m, c->doc_off_h[d + 1] - c->doc_off_h[d]);
  *max_len = (int32_t)m;
  return LDA_OK;
  });
}

lda_status lda_doc_topic_histograms(lda_ctx* c, int32_t max_len, int32_t* doc_len_counts,
                                    int32_t* topic_doc_counts) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !doc_len_counts || !topic_doc_counts) return fail(LDA_ERR_INVALID_ARG, "null argument");
  int32_t m = 0;
  lda_max_doc_length(c, &m);
  if (max_len < m) return fail(LDA_ERR_INVALID_ARG, "max_len below the longest document");
  if (c->pending) return fail(LDA_ERR_STATE, "histograms with a pending delta: call lda_apply first");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t L1 = (int64_t)max_len + 1;
  const size_t n = (size_t)L1 + (size_t)c->K * L1;
  int32_t* buf = nullptr;
  HIP_TRY(dalloc(&buf, n));
  std::vector<int32_t> h;
  try {
    h = host_vector<int32_t>(n);
  } catch (...) {
    (void)hipFree(buf);
    throw;
  }
  hipError_t e = hipMemsetAsync(buf, 0, n * sizeof(int32_t), c->stream);
  if (e == hipSuccess)
    e = lda::launch_doc_hist(c->z, c->doc_off, c->D, c->K, c->Kp, max_len, buf, buf + L1, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), buf, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(buf);
  HIP_TRY(e);
  for (int64_t i = 0; i < L1; ++i) doc_len_counts[i] += h[i];
  for (size_t i = 0; i < (size_t)c->K * L1; ++i) topic_doc_counts[i] += h[L1 + i];
  return LDA_OK;
  });
}

lda_status lda_doc_topic_histograms_accumulate(lda_ctx* c, int32_t max_len) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  int32_t m = 0;
  lda_max_doc_length(c, &m);
  if (max_len < m) return fail(LDA_ERR_INVALID_ARG, "max_len below the longest document");
  if (c->pending) return fail(LDA_ERR_STATE, "histograms with a pending delta: call lda_apply first");
  if (c->stat_buf && c->stat_len != max_len)
    return fail(LDA_ERR_STATE, "max_len differs from the accumulated histograms': take them first");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t L1 = (int64_t)max_len + 1;
  const size_t n = (size_t)L1 + (size_t)c->K * L1;
  if (!c->stat_buf) {
    HIP_TRY(dalloc(&c->stat_buf, n));
    HIP_TRY(hipMemsetAsync(c->stat_buf, 0, n * sizeof(int32_t), c->stream));
    c->stat_len = max_len;
  }
  HIP_TRY(lda::launch_doc_hist(c->z, c->doc_off, c->D, c->K, c->Kp, max_len, c->stat_buf, c->stat_buf + L1,
                               c->stream));
  return LDA_OK;
  });
}

lda_status lda_doc_topic_histograms_take(lda_ctx* c, int32_t max_len, int32_t* doc_len_counts,
                                         int32_t* topic_doc_counts) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !doc_len_counts || !topic_doc_counts) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (!c->stat_buf) return LDA_OK;           // nothing accumulated
  if (c->stat_len != max_len) return fail(LDA_ERR_INVALID_ARG, "max_len differs from the accumulated histograms'");
  HIP_TRY(hipSetDevice(c->device));
  const int64_t L1 = (int64_t)max_len + 1;
  const size_t n = (size_t)L1 + (size_t)c->K * L1;
  std::vector<int32_t> h = host_vector<int32_t>(n);
  HIP_TRY(hipMemcpyAsync(h.data(), c->stat_buf, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemsetAsync(c->stat_buf, 0, n * sizeof(int32_t), c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  for (int64_t i = 0; i < L1; ++i) doc_len_counts[i] += h[(size_t)i];
  for (size_t i = 0; i < (size_t)c->K * L1; ++i) topic_doc_counts[i] += h[L1 + i];
  return LDA_OK;
  });
}

lda_status lda_doc_topic_histograms_clear(lda_ctx* c) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if (!c->stat_buf) return LDA_OK;
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)(c->stat_len + 1) * (size_t)(c->K + 1);
  HIP_TRY(hipMemsetAsync(c->stat_buf, 0, n * sizeof(int32_t), c->stream));
  return LDA_OK;
  });
}

lda_status lda_count_histogram(lda_ctx* c, int64_t max_count, int32_t* count_hist) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !count_hist || max_count < 0) return fail(LDA_ERR_INVALID_ARG, "bad argument");
  if (c->pending) return fail(LDA_ERR_STATE, "histogram with a pending delta: call lda_apply first");
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)max_count + 1;
  if (c->chist_cap < n + 1) {
    if (c->chist) (void)hipFree(c->chist);
    c->chist = nullptr;
    c->chist_cap = 0;
    HIP_TRY(dalloc(&c->chist, n + 1));
    c->chist_cap = n + 1;
  }
  int32_t* buf = c->chist;
  std::vector<int32_t> h = host_vector<int32_t>(n + 1);
  HIP_TRY(hipMemsetAsync(buf, 0, (n + 1) * sizeof(int32_t), c->stream));
  HIP_TRY(lda::launch_count_hist(c->nw, c->V, c->K, c->Kp, max_count, buf, buf + n, c->stream));
  HIP_TRY(hipMemcpyAsync(h.data(), buf, (n + 1) * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  if (h[n]) return fail(LDA_ERR_INVALID_ARG, "an nw cell exceeds max_count");
  for (size_t i = 0; i < n; ++i) count_hist[i] += h[i];
  return LDA_OK;
  });
}

lda_status lda_hyper_statistics(lda_ctx* c, int32_t max_len, int32_t* doc_len_counts, int32_t* topic_doc_counts,
                                int64_t max_count, int32_t* count_hist, int32_t* nwsum) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c) return fail(LDA_ERR_INVALID_ARG, "null ctx");
  if ((doc_len_counts == nullptr) != (topic_doc_counts == nullptr))
    return fail(LDA_ERR_INVALID_ARG, "doc_len_counts and topic_doc_counts go together");
  if (count_hist && max_count < 0) return fail(LDA_ERR_INVALID_ARG, "max_count must be >= 0");
  if (c->pending && (count_hist || nwsum)) return fail(LDA_ERR_STATE, "statistics with a pending delta: call lda_apply first");
  const bool docs = doc_len_counts && c->stat_buf;
  if (docs && c->stat_len != max_len) return fail(LDA_ERR_INVALID_ARG, "max_len differs from the accumulated histograms'");
  HIP_TRY(hipSetDevice(c->device));
  const size_t L1 = (size_t)max_len + 1;
  const size_t n_doc = docs ? L1 + (size_t)c->K * L1 : 0;
  const size_t n_cnt = count_hist ? (size_t)max_count + 2 : 0;   // + the overflow cell
  const size_t n_sum = nwsum ? (size_t)c->K : 0;
  const size_t need = n_doc + n_cnt + n_sum;
  if (need == 0) return LDA_OK;
  if (c->hyper_pin_cap < need) {
    if (c->hyper_pin) (void)hipHostFree(c->hyper_pin);
    c->hyper_pin = nullptr;
    c->hyper_pin_cap = 0;
    HIP_TRY(hipHostMalloc(&c->hyper_pin, sizeof(int32_t) * need, hipHostMallocDefault));
    c->hyper_pin_cap = need;
  }
  int32_t* h = c->hyper_pin;
  if (docs) {
    HIP_TRY(hipMemcpyAsync(h, c->stat_buf, n_doc * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemsetAsync(c->stat_buf, 0, n_doc * sizeof(int32_t), c->stream));
  }
  if (count_hist) {
    if (c->chist_cap < n_cnt) {
      if (c->chist) (void)hipFree(c->chist);
      c->chist = nullptr;
      c->chist_cap = 0;
      HIP_TRY(dalloc(&c->chist, n_cnt));
      c->chist_cap = n_cnt;
    }
    HIP_TRY(hipMemsetAsync(c->chist, 0, n_cnt * sizeof(int32_t), c->stream));
    HIP_TRY(lda::launch_count_hist(c->nw, c->V, c->K, c->Kp, max_count, c->chist, c->chist + n_cnt - 1, c->stream));
    HIP_TRY(hipMemcpyAsync(h + n_doc, c->chist, n_cnt * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  }
  if (nwsum)
    HIP_TRY(hipMemcpyAsync(h + n_doc + n_cnt, c->nwsum, n_sum * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));   // the one wait
  if (count_hist && h[n_doc + n_cnt - 1]) return fail(LDA_ERR_INVALID_ARG, "an nw cell exceeds max_count");
  for (size_t i = 0; i < n_doc; ++i) (i < L1 ? doc_len_counts[i] : topic_doc_counts[i - L1]) += h[i];
  for (size_t i = 0; i + 1 < n_cnt; ++i) count_hist[i] += h[n_doc + i];
  for (size_t i = 0; i < n_sum; ++i) nwsum[i] = h[n_doc + n_cnt + i];
  return LDA_OK;
  });
}

lda_status lda_row_stats(lda_ctx* c, double* mean_row_nnz) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !mean_row_nnz) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (c->pending) return fail(LDA_ERR_STATE, "row statistics with a pending delta: call lda_apply first");
  HIP_TRY(hipSetDevice(c->device));
  unsigned long long* buf = nullptr;
  HIP_TRY(dalloc(&buf, 2));
  unsigned long long h[2] = {0, 0};
  hipError_t e = hipMemsetAsync(buf, 0, 2 * sizeof(unsigned long long), c->stream);
  if (e == hipSuccess) e = lda::launch_row_stats(c->nw, c->V, c->K, c->Kp, buf, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(h, buf, sizeof(h), hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(buf);
  HIP_TRY(e);
  *mean_row_nnz = h[1] ? (double)h[0] / (double)h[1] : 0.0;
  return LDA_OK;
  });
}

lda_status lda_infer(lda_ctx* c, int64_t Dh, const int64_t* doc_off, const int32_t* words_in,
                     int32_t n_iter, int32_t thin, int32_t burn_in, uint64_t seed, double* theta) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !doc_off || !theta) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (Dh < 0 || n_iter < 0 || burn_in < 0 || thin < 1) return fail(LDA_ERR_INVALID_ARG, "bad sizes");
  if (c->pending) return fail(LDA_ERR_STATE, "inference with a pending delta: call lda_apply first");
  for (int64_t d = 1; d <= Dh; ++d)
    if (doc_off[d] < doc_off[d - 1]) return fail(LDA_ERR_INVALID_ARG, "doc_off not monotone");
  const int64_t N_in = doc_off[Dh] - doc_off[0];
  if (N_in > 0 && !words_in) return fail(LDA_ERR_INVALID_ARG, "words is null");
  for (int64_t i = 0; i < N_in; ++i)
    if (words_in[i] < 0 || words_in[i] >= c->V) return fail(LDA_ERR_INVALID_ARG, "word id out of range (OOV must be removed)");
  HIP_TRY(hipSetDevice(c->device));
  // TopicInferencer skips tokens whose type has no training tokens (an empty
  // typeTopicCounts row): drop them here (row totals of the global snapshot,
  // computed once per snapshot)
  if (c->totals_gen != c->apply_gen) {
    int32_t* caps = nullptr;
    HIP_TRY(dalloc(&caps, c->V));
    c->word_totals.assign((size_t)c->V, 0);
    hipError_t e = lda::launch_row_caps(c->nw, c->V, c->Kp, caps, c->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(c->word_totals.data(), caps, sizeof(int32_t) * c->V, hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(caps);
    HIP_TRY(e);
    c->totals_gen = c->apply_gen;
  }
  std::vector<int64_t> off(Dh + 1);
  std::vector<int32_t> kept;
  kept.reserve((size_t)N_in);
  off[0] = 0;
  for (int64_t d = 0; d < Dh; ++d) {
    for (int64_t i = doc_off[d] - doc_off[0]; i < doc_off[d + 1] - doc_off[0]; ++i)
      if (c->word_totals[(size_t)words_in[i]] > 0) kept.push_back(words_in[i]);
    off[d + 1] = (int64_t)kept.size();
  }
  const int32_t* words = kept.data();
  const int64_t N = off[Dh];
  if (c->Kp > 1024)
    for (int64_t d = 0; d < Dh; ++d)
      if (off[d + 1] - off[d] > LDA_MAX_DOC_TOKENS_BIGK)
        return fail(LDA_ERR_UNSUPPORTED, "document longer than 65535 tokens with num_topics > 1024");
  std::vector<int64_t> ranges = make_ranges(off, std::max<int64_t>(16, std::min<int64_t>(c->tokens_per_range, N / std::max<int64_t>(1, (int64_t)c->sample_blocks_frozen * c->waves_per_block * 8))));
  const int64_t R = (int64_t)ranges.size() - 1;
  hipError_t e = hipSuccess;
  auto chk = [&](hipError_t x) {
    if (e == hipSuccess) e = x;
  };
  // grow-only scratch (kept by the context between calls)
  auto need = [&](auto*& ptr, size_t n, int slot) {
    if (e != hipSuccess || n <= c->inf_cap[slot]) return;
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    c->inf_cap[slot] = 0;
    chk(dalloc(&ptr, n));
    if (e == hipSuccess) c->inf_cap[slot] = n;
  };
  need(c->inf_words, (size_t)std::max<int64_t>(N, 1), 0);
  need(c->inf_z, (size_t)std::max<int64_t>(N, 1), 1);
  need(c->inf_acc, (size_t)std::max<int64_t>(Dh, 1) * c->K, 2);
  need(c->inf_q, (size_t)std::max<int32_t>(n_iter, 1), 3);   // one work-queue counter per iteration
  need(c->inf_doff, (size_t)Dh + 1, 4);
  need(c->inf_range, ranges.size(), 5);
  int32_t *dw = c->inf_words, *dz = c->inf_z, *acc = c->inf_acc, *q = c->inf_q;
  int64_t *doff = c->inf_doff, *drange = c->inf_range;
  if (e == hipSuccess && N > 0) chk(hipMemcpyAsync(dw, words, sizeof(int32_t) * N, hipMemcpyHostToDevice, c->stream));
  if (e == hipSuccess) chk(hipMemcpyAsync(doff, off.data(), sizeof(int64_t) * (Dh + 1), hipMemcpyHostToDevice, c->stream));
  if (e == hipSuccess) chk(hipMemcpyAsync(drange, ranges.data(), sizeof(int64_t) * ranges.size(), hipMemcpyHostToDevice, c->stream));
  if (e == hipSuccess) chk(hipMemsetAsync(acc, 0, sizeof(int32_t) * (size_t)std::max<int64_t>(Dh, 1) * c->K, c->stream));
  if (e == hipSuccess) chk(hipMemsetAsync(q, 0, sizeof(int32_t) * (size_t)std::max<int32_t>(n_iter, 1), c->stream));
  if (e == hipSuccess) chk(lda::launch_infer_init(dw, dz, N, c->nw, c->K, c->Kp, c->stream));
  int32_t nsamples = 0;
  lda::SampleParams p = c->params(true);
  p.words = dw;
  p.z = dz;
  p.doc_off = doff;
  p.range_doc = drange;
  p.range_end = drange + 1;
  p.num_ranges = R;
  p.delta = nullptr;
  p.dsum = nullptr;
  p.token_base = 0;
  p.k0 = (uint32_t)seed;
  p.k1 = (uint32_t)(seed >> 32);
  p.c3 = lda::STREAM_INFER;
  const int64_t wpb = c->waves_per_block;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(c->sample_blocks_frozen, (R + wpb - 1) / wpb));
  for (int32_t it = 1; it <= n_iter && e == hipSuccess && N > 0; ++it) {
    p.c2 = (uint32_t)(it - 1);
    p.queue = q + (it - 1);
    chk(c->sampler == LDA_SAMPLER_SPARSE ? lda::launch_sample_sparse(c->C, true, p, blocks, c->stream)
                                         : lda::launch_sample(c->C, true, p, blocks, c->stream, c->half));
    if (it > burn_in && (it - burn_in) % thin == 0) {
      ++nsamples;
      if (e == hipSuccess) chk(lda::launch_doc_topics(dz, doff, Dh, c->K, c->Kp, acc, 1, c->stream));
    }
  }
  if (nsamples == 0) {
    nsamples = 1;
    if (e == hipSuccess) chk(lda::launch_doc_topics(dz, doff, Dh, c->K, c->Kp, acc, 1, c->stream));
  }
  std::vector<int32_t> acc_h = host_vector<int32_t>((size_t)Dh * c->K);
  if (e == hipSuccess && Dh > 0)
    chk(hipMemcpyAsync(acc_h.data(), acc, sizeof(int32_t) * (size_t)Dh * c->K, hipMemcpyDeviceToHost, c->stream));
  if (e == hipSuccess) chk(hipStreamSynchronize(c->stream));
  HIP_TRY(e);
  for (int64_t d = 0; d < Dh; ++d) {
    double sum = 0.0;
    for (int k = 0; k < c->K; ++k) {
      const double v = (double)nsamples * c->alpha[k] + (double)acc_h[(size_t)d * c->K + k];
      theta[(size_t)d * c->K + k] = v;
      sum += v;
    }
    for (int k = 0; k < c->K; ++k) theta[(size_t)d * c->K + k] /= sum;
  }
  return LDA_OK;
  });
}

lda_status lda_to_mallet_packed(lda_ctx* c, int32_t* rows, int64_t* row_off, int32_t* topic_bits) {
  return lda_abi::guarded([&]() -> lda_status {
  if (!c || !row_off) return fail(LDA_ERR_INVALID_ARG, "null argument");
  if (c->pending) return fail(LDA_ERR_STATE, "pending delta: call lda_apply first");
  // ParallelTopicModel(numberOfTopics, ...): topicMask / topicBits [M]
  int32_t mask;
  if ((c->K & (c->K - 1)) == 0) {
    mask = c->K - 1;
  } else {
    int hb = 1;
    while (hb * 2 <= c->K) hb *= 2;
    mask = hb * 2 - 1;
  }
  const int32_t bits = __builtin_popcount((unsigned)mask);
  if (topic_bits) *topic_bits = bits;
  std::vector<int32_t> nw = host_vector<int32_t>((size_t)c->V * c->K);
  lda_status s = lda_get_counts(c, nw.data(), nullptr, nullptr, nullptr);
  if (s) return s;
  // row length = min(K, typeTotal) exactly as addInstances allocates it
  row_off[0] = 0;
  for (int w = 0; w < c->V; ++w) {
    int64_t total = 0;
    for (int k = 0; k < c->K; ++k) total += nw[(size_t)w * c->K + k];
    row_off[w + 1] = row_off[w] + std::min<int64_t>(c->K, total);
  }
  if (!rows) return LDA_OK;
  std::vector<int32_t> cell;
  for (int w = 0; w < c->V; ++w) {
    cell.clear();
    for (int k = 0; k < c->K; ++k) {
      const int32_t n = nw[(size_t)w * c->K + k];
      if (n > 0) {
        if ((int64_t)n >= (1LL << (31 - bits)))
          return fail(LDA_ERR_UNSUPPORTED, "count does not fit Mallet's packed cell");
        cell.push_back((n << bits) + k);
      }
    }
    std::sort(cell.begin(), cell.end(), [](int32_t a, int32_t b) { return a > b; });
    int64_t o = row_off[w];
    const int64_t len = row_off[w + 1] - row_off[w];
    for (int64_t i = 0; i < len; ++i) rows[o + i] = i < (int64_t)cell.size() ? cell[i] : 0;
  }
  return LDA_OK;
  });
}

}  // extern "C"
