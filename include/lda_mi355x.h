/*
 * lda_mi355x.h — C ABI of the MI355X-native collapsed-Gibbs LDA sampler.
 *
 * This is the drop-in boundary for the reference's only hot path: the
 * per-token z-resampling loop that qianjinding/LDAGibbsSampling delegates to
 * Mallet 2.0.7 (pom.xml:107-111) through
 *     ParallelTopicModel.estimate()            src/cmu_ron/TrainAndPredict.java:166
 *                                              src/cmu/TrainAndPredict.java:265
 * and from there WorkerRunnable.sampleTopicsForOneDoc (Mallet, not vendored).
 * The reference has no FFI of its own; the seam is Mallet's public class API
 * as called from trainNewModel (src/cmu_ron/TrainAndPredict.java:159-171,
 * src/cmu/TrainAndPredict.java:258-269).  Each entry point below names the
 * Mallet call it replaces; INTEGRATION.md shows the JNI binding a Java
 * maintainer adds (GpuParallelTopicModel extends ParallelTopicModel).
 *
 * Conventions
 *  - Plain pointers and sizes only.  The caller owns every host buffer;
 *    lda_create copies its inputs into device memory and no pointer is kept
 *    after a call returns (except lda_delta_buffer's device pointer, which is
 *    owned by the context).
 *  - Every call returns an lda_status (0 = OK, < 0 = error class);
 *    lda_last_error() gives a thread-local message.  No C++ exception crosses
 *    the ABI.
 *  - One context = one GPU = one caller thread (not re-entrant per context).
 *    Multi-GPU: one process (or thread) per GPU, each with a context over its
 *    own document shard, exchanging the nw/nwsum delta buffer with an
 *    all-reduce between lda_sample() and lda_apply() (AD-LDA).
 *  - Counts are int32 (exact).  Sampling weights are fp32, evaluated in the
 *    fixed order documented in DESIGN.md so that z/nw/nwsum/nd are bit-exact
 *    against the CPU oracle and independent of GPU count and scheduling.
 */
#ifndef LDA_MI355X_H
#define LDA_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t lda_status;
#define LDA_OK 0
#define LDA_ERR_INVALID_ARG (-1)
#define LDA_ERR_DEVICE (-2)       /* HIP runtime / kernel launch failure */
#define LDA_ERR_OUT_OF_MEMORY (-3)
#define LDA_ERR_STATE (-4)        /* call out of order (e.g. sample with a pending delta) */
#define LDA_ERR_UNSUPPORTED (-5)  /* e.g. K above the compiled maximum */
#define LDA_ERR_INTERNAL (-6)     /* an unexpected C++ exception, caught at the ABI */

#define LDA_MAX_TOPICS 4096       /* K <= 4096 (LDA_SAMPLER_SPARSE above 1024)       */
#define LDA_MAX_TOPICS_DENSE 1024 /* the dense sampler's register-resident rows      */
/* With K > 1024 (Kp > 1024) a document's topic counts live in LDS as 16-bit
 * pairs: documents are limited to 65535 tokens there (LDA_ERR_UNSUPPORTED). */
#define LDA_MAX_DOC_TOKENS_BIGK 65535

/* Draw kernels.  Both are exact against the CPU oracle.
 *  DENSE   reads the word's whole row from a 16-bit copy of nw (2K bytes per
 *          token; the int32 row for words with a count > 65535);
 *  SPARSE  reads only the row's nonzero (count, topic) entries (4 bytes each),
 *          SparseLDA-style split into a word part and a dense doc part
 *          (a different fp32 summation with its own oracle restatement). */
/* The dense sampler needs num_types * Kp < 2^32 (V < 4.19M words at K = 1024). */
#define LDA_SAMPLER_DENSE 0
#define LDA_SAMPLER_SPARSE 1

typedef struct lda_ctx lda_ctx;

typedef struct lda_config {
  int32_t num_topics;     /* K      (ParallelTopicModel(numberOfTopics, ...)) */
  int32_t num_types;      /* V      (alphabet size; word ids are 0..V-1)       */
  int64_t num_docs;       /* D      documents in THIS shard                    */
  const double* alpha;    /* [K] per-topic alpha (alphaSum/K when symmetric)   */
  double beta;            /* beta   (ParallelTopicModel(.., .., beta))         */
  uint64_t seed;          /* Philox key (ParallelTopicModel.setRandomSeed)     */
  int32_t device;         /* HIP device ordinal                                */
  int32_t sampler;        /* LDA_SAMPLER_DENSE (0) or LDA_SAMPLER_SPARSE (1)   */
  int64_t token_base;     /* global index of this shard's first token          */
  int64_t tokens_per_range; /* work-queue granule (0 = default)                */
} lda_config;

/* Create a sampler over one shard.  doc_off[D+1] (int64, doc_off[0] may be
 * non-zero: offsets are rebased), words[N] (int32 word ids), z_init[N] or NULL
 * (NULL = Philox initialisation, the GPU analogue of addInstances' random
 * topics).  The shard's own counts are left as the PENDING delta: call
 * lda_apply (after an all-reduce of lda_delta_buffer when sharded) before the
 * first lda_sample.  Replaces ParallelTopicModel(K, alphaSum, beta) +
 * addInstances(InstanceList)  [src/cmu_ron/TrainAndPredict.java:160-162]. */
lda_status lda_create(lda_ctx** out, const lda_config* cfg, const int64_t* doc_off,
                      const int32_t* words, const int32_t* z_init);
void lda_destroy(lda_ctx* ctx);

/* Run n full sweeps on a single (unsharded) context: apply any pending delta,
 * then n x (sample + apply).  Replaces ParallelTopicModel.estimate() with
 * setNumIterations(n) and optimizeInterval 0 [src/cmu_ron/TrainAndPredict.java:165-166].
 * Plain dense sweeps (one part, not warm-start or recount sweeps) are
 * launched as hipGraphs of up to 16 sweeps, captured once per length on the
 * context's stream; the results are those of n lda_sample + lda_apply calls
 * (the sweep counter and beta are read from device memory).  No event timing
 * is recorded for them (lda_sample_times covers lda_sample launches).  The
 * environment variable LDA_GRAPHS=0 at lda_create turns the graphs off. */
lda_status lda_sweep(lda_ctx* ctx, int32_t n);

/* One sampling pass over the shard against the current nw/nwsum snapshot
 * (one sweep of WorkerRunnable.run()); its result goes to the exchange
 * buffer below.  Asynchronous on the context's stream, except that the
 * large-K sampler (K > 1024) times its two ring depths from the ninth sweep
 * on, every 19 sweeps: the sweep after such a probe waits on the host for
 * the probe's last launch (LDA_SB_RB=short or default at
 * lda_create fixes the ring and never waits).  Either ring gives the same
 * draws. */
lda_status lda_sample(lda_ctx* ctx);
/* Device pointer to the pending exchange buffer: int32[V*Kp + Kp] (an nw part
 * row-major with padded row length Kp = lda_padded_topics(), then an nwsum
 * part).  Sum it across ranks in place (the sumTypeTopicCounts analogue)
 * before lda_apply.  What it holds depends on the count-update mode
 * (lda_count_update_mode): the dense samplers RECOUNT -- the sampler writes
 * only z and the buffer receives this shard's own (word, topic) counts, which
 * lda_apply's sum replaces nw / nwsum with -- the sparse samplers keep a
 * DELTA of the shard's changes, which lda_apply adds.  Either way the caller
 * only sums it, and lda_apply leaves it zero. */
lda_status lda_delta_buffer(lda_ctx* ctx, void** dev_ptr, size_t* count);
/* recount = 1 when the pending buffer holds counts (or, with nothing
 * pending, when the next sweep will recount), 0 for a delta. */
lda_status lda_count_update_mode(lda_ctx* ctx, int32_t* recount);
/* Which sweeps recount (dense samplers; the sparse ones always keep a delta).
 *  LDA_COUNT_AUTO     the first recount_sweeps sweeps after the counts are
 *                     (re)seeded by lda_create / lda_set_z recount, later
 *                     ones keep a delta (near init nearly every token
 *                     changes, and the delta's device atomics cost more than
 *                     the recount; later they cost less).  The default is
 *                     LDA_RECOUNT_SWEEPS_DEFAULT when K <= 128 and the
 *                     shard holds 2^20 <= N tokens with z fitting the
 *                     Infinity Cache (4 N <= 256 MiB), else 0 (measured
 *                     crossover: DESIGN.md §4).
 *                     recount_sweeps < 0 keeps the current value.
 *                     Sequential sweeps -- warm-start sweeps
 *                     (lda_set_warm_start) and the steady ones of
 *                     lda_set_sequential_sweeps -- never recount under AUTO
 *                     but do count toward the window: with the native
 *                     ParallelTopicModel's default 4 x 50 warm start the
 *                     window has passed before the first plain sweep, which
 *                     is right, since after ~20 sweeps the delta is the
 *                     faster update; and its default Mallet-
 *                     staleness schedule makes every later sweep sequential
 *                     as well.  AUTO recount therefore acts only on plain
 *                     snapshot sweeps (lda_sweep without either schedule,
 *                     bench.py).
 *  LDA_COUNT_RECOUNT  every sweep, sequential ones included (after each part
 *                     the whole shard is recounted into buffer 0, the parts
 *                     sampled so far with their new topics);
 *  LDA_COUNT_DELTA    none.
 * Shards exchanging buffers must agree on it sweep by sweep: a distributed
 * driver sets the same mode and count on every rank (ADLDATrainer: the
 * minimum over ranks).  Results are identical in every mode.  On recount
 * sweeps the K <= 128 default sampler also keeps a copy of z in the
 * recount's word order (N int32 + N uint32 of device memory, allocated at
 * the first recount sweep) so that the recount streams it instead of
 * gathering z; LDA_ZW=0 at lda_create turns the copy off. */
#define LDA_COUNT_AUTO 0
#define LDA_COUNT_RECOUNT 1
#define LDA_COUNT_DELTA 2
#define LDA_RECOUNT_SWEEPS_DEFAULT 20
lda_status lda_set_count_update(lda_ctx* ctx, int32_t mode, int32_t recount_sweeps);
lda_status lda_get_count_update(lda_ctx* ctx, int32_t* mode, int32_t* recount_sweeps);
/* nw/nwsum := buffer (recount) or += buffer (delta), buffer = 0, refresh the
 * per-topic tables. */
lda_status lda_apply(lda_ctx* ctx);

/* Split sweep: the exchange overlapped with sampling.
 * Mallet sums its workers' counts only after every worker has finished the
 * sweep (ParallelTopicModel.sumTypeTopicCounts, [M]); here the shard's work
 * ranges are cut into `parts` token-balanced parts (1..LDA_MAX_EXCHANGE_PARTS),
 * each with its own delta buffer.  lda_sample_part(ctx, i) samples part i
 * against the unchanged snapshot; after it, buffer i is final for the sweep,
 * so its all-reduce can run (on another stream) while part i+1 samples.
 * Parts are sampled in order 0..parts-1 and all use the same sweep counter;
 * lda_apply folds every buffer.  Results are identical for any `parts`
 * (integer sums; draws keyed by the global token index).  lda_sample runs
 * every part.  reserve_cus: CUs' worth of sampler blocks left free in a split
 * sweep for the collective's kernels (0 = none, < 0 = the default: 1/32 of
 * the device's CUs, 8 on MI355X).  Sequential sweeps (warm start, steady
 * schedule) ignore the split: their parts are the schedule's, each summed and
 * applied before the next part samples (an exchange per part, nothing to
 * overlap), so under the native ParallelTopicModel's default staleness
 * schedule a multi-GPU sweep exchanges 2-4 times. */
#define LDA_MAX_EXCHANGE_PARTS 4
lda_status lda_set_exchange_parts(lda_ctx* ctx, int32_t parts, int32_t reserve_cus);
lda_status lda_get_exchange_parts(lda_ctx* ctx, int32_t* parts);
lda_status lda_sample_part(lda_ctx* ctx, int32_t part);
lda_status lda_delta_buffer_part(lda_ctx* ctx, int32_t part, void** dev_ptr, size_t* count);

/* Compact exchange.  The buffer of lda_delta_buffer_part
 * holds int32 cells [V*Kp | Kp]; summed across `world` ranks as they are,
 * that is 4 (V Kp + Kp) bytes per sweep (C5: 4.3 GB).  Instead a driver may
 * exchange it packed, two cells per int32 word:
 *   lda_exchange_sizes: packed_count int32 words [V*Kp/2 | Kp] and
 *     escape_count int32 of one rank's escape list, for `world` ranks whose
 *     largest shard holds max_shard_tokens tokens (the same on every rank);
 *   lda_exchange_pack(part): packs the part's buffer on the context's stream
 *     and returns the context-owned device arrays to exchange;
 *   the driver: SUM all-reduce (int32) of `packed` in place, and an
 *     all-gather of every rank's `escapes` into one device array
 *     [world x escape_count] in rank order;
 *   lda_exchange_unpack(part, escapes_all): the part's buffer = the unpacked
 *     sum plus every rank's escapes (then lda_apply as usual).
 * Cell 2i packs as d + 2^15/world (bits 0..15), cell 2i+1 as d + 2^14/world
 * (bits 16..30): the sum over the ranks cannot carry between the halves or
 * overflow int32.  Cells outside that range travel in the escape list
 * (count, then (cell lo, cell hi, value) triples); each rank has at most
 * 2 max_shard_tokens / (2^14/world) of them, since a rank's |cells| sum to
 * at most twice its tokens.  The result is the int32 sum, bit for bit. */
lda_status lda_exchange_sizes(lda_ctx* ctx, int32_t world, int64_t max_shard_tokens, size_t* packed_count,
                              size_t* escape_count);
lda_status lda_exchange_pack(lda_ctx* ctx, int32_t part, int32_t world, int64_t max_shard_tokens, void** packed,
                             void** escapes);
lda_status lda_exchange_unpack(lda_ctx* ctx, int32_t part, int32_t world, int64_t max_shard_tokens,
                               const void* escapes_all);
/* The escape lists sent at their used length (ldagibbssampling_amd/
 * distributed.py): escapes[0] after lda_exchange_pack is the rank's escape
 * count n (n > escape capacity cannot happen when every rank's shard holds at
 * most max_shard_tokens tokens; a driver that reads n > capacity must stop).
 * A driver that MAX-all-reduces n into m (identical on every rank) may
 * all-gather only the first 1 + 3 m int32 of each rank's list into
 * [world x (1 + 3 m)] and unpack with list_cap = m; m = 0 needs no all-gather
 * (escapes_all may be NULL).  list_cap in [0, capacity]; lda_exchange_unpack
 * is list_cap = capacity. */
lda_status lda_exchange_unpack_lists(lda_ctx* ctx, int32_t part, int32_t world, int64_t max_shard_tokens,
                                     const void* escapes_all, int32_t list_cap);
/* Cells per packed word (round 6): 2 (the default, above) or 4 -- cells
 * 4i..4i+2 as d + 2^7/world in bits 0..7, 8..15, 16..23 and cell 4i+3 as
 * d + 2^6/world in bits 24..30 (world <= 64), half the packed bytes of the
 * default (C5 at 8 ranks: 1.07 GB instead of 2.15 GB per exchange) at the
 * price of more escapes (a cell escapes beyond [-16, 16) at 8 ranks instead
 * of [-2048, 2048)); the escape capacity of lda_exchange_sizes follows the
 * smaller bias.  Every rank of a group must use the same value.  The result
 * is the same int32 sum, bit for bit. */
lda_status lda_set_exchange_cells(lda_ctx* ctx, int32_t cells_per_word);
lda_status lda_get_exchange_cells(lda_ctx* ctx, int32_t* cells_per_word);
/* Replica check (bench.py's multi-GPU line): a hash of the applied counts,
 * the sum mod 2^64 over the nonzero cells of nw (V x K) and nwsum (K) of
 * splitmix64's finaliser applied to (index << 32 | (uint32)value), index =
 * w K + k in nw and V K + k in nwsum (oracle.counts_checksum).  Every rank of
 * an AD-LDA group holds the same replica, so MIN == MAX over the ranks.
 * LDA_ERR_STATE with a pending delta.  Synchronises the context's stream. */
lda_status lda_counts_checksum(lda_ctx* ctx, uint64_t* checksum);

/* Warm start.  The GPU sweep samples every document against one snapshot
 * (AD-LDA), while Mallet's setNumThreads(4) workers each see their own
 * changes live: from a random start the snapshot sweep falls into a local
 * optimum more often (held-out perplexity over 96 seeds at
 * K = 20).  With lda_set_warm_start(ctx, parts, sweeps) the sweeps whose
 * sweep counter (lda_get_sweep: carried across estimate() calls and
 * checkpoints) is below `sweeps` run in `parts` token-balanced parts in
 * SEQUENTIAL order: part i samples against
 * the snapshot with parts 0..i-1 of this sweep applied.  Such a sweep keeps
 * its changes in buffer 0 (lda_delta_buffer_part returns it for every part)
 * and is never a recount sweep.  lda_sample / lda_sweep do it by themselves;
 * a sharding driver asks lda_sweep_parts and, when sequential, runs for
 * each part: lda_sample_part(i), sum buffer 0 across ranks, lda_apply.
 * parts in [1, LDA_MAX_EXCHANGE_PARTS] (1 = off).  The parts are cut in
 * the whole corpus, global token indices [corpus_first_token,
 * corpus_first_token + corpus_tokens) (corpus_tokens <= 0: this shard is the
 * whole corpus), into S = parts * LDA_WARM_BLOCKS token-balanced segments:
 * cut j is the first document starting at or after token
 * first + tokens * j / S, and segment j belongs to part j % parts.  A shard
 * samples its own documents of global part i in step i, so the result is the
 * same for any sharding and identical to cpu_exact's same schedule, and every
 * shard of a token-balanced sharding into <= LDA_WARM_BLOCKS shards has work
 * in every step. */
#define LDA_WARM_BLOCKS 64
/* Sequential parts are cut at cumulative fractions of each block in units of
 * 1 / LDA_SEQ_FRACTION_UNIT (lcm(1..16): equal parts are exact). */
#define LDA_SEQ_FRACTION_UNIT 720720
/* Host-only (no device call): the tokens a shard (documents doc_off[0..D],
 * global token base + doc_off[d] - doc_off[0]) samples in each warm-start
 * part of the corpus [corpus_first_token, + corpus_tokens), as
 * lda_set_warm_start cuts them; tokens_out[parts]. */
lda_status lda_warm_part_tokens(const int64_t* doc_off, int64_t num_docs, int32_t parts, int64_t token_base,
                                int64_t corpus_first_token, int64_t corpus_tokens, int64_t* tokens_out);
lda_status lda_set_warm_start(lda_ctx* ctx, int32_t parts, int32_t sweeps, int64_t corpus_first_token,
                              int64_t corpus_tokens);
lda_status lda_get_warm_start(lda_ctx* ctx, int32_t* parts, int32_t* sweeps);
/* Steady sequential sweeps: Mallet's staleness.  The snapshot sweep shows
 * every token none of the sweep's other changes; Mallet's setNumThreads(T)
 * workers each see their own changes live, so a token sees on average
 * 1/(2T) of them.  That difference is measurable at the reference's own
 * training settings: with hyperparameter optimisation the snapshot sweep
 * learns beta ~9% higher and alphaSum ~4% lower than Mallet's 4 threads and,
 * at K = 500, traps more chains.
 * lda_set_sequential_sweeps(ctx, parts, fractions, first, tokens): every
 * sweep that is not a warm-start sweep runs in `parts` sequential parts (as
 * the warm start's, each applied before the next samples, all through buffer
 * 0), part i taking the fraction fractions[i] of each of the
 * LDA_WARM_BLOCKS blocks of the corpus (fractions NULL: equal parts); parts
 * = 1 turns it off (the default: lda_sweep's plain snapshot sweeps).  The
 * corpus arguments are lda_set_warm_start's.  lda_staleness_schedule(T)
 * gives the schedule with Mallet's mean live fraction for T threads: two
 * parts, the first f = (1 - sqrt(1 - 2/T)) / 2 of every block (T = 4: f =
 * 0.146), so that f (1 - f) = 1/(2T); T = 1 gives LDA_MAX_EXCHANGE_PARTS
 * equal parts (mean 3/8, the nearest to sequential Mallet's 1/2).
 * lda_get_sequential_sweeps: the parts and the cumulative cut fractions
 * cum_units[parts + 1] in units of 1 / LDA_SEQ_FRACTION_UNIT. */
lda_status lda_set_sequential_sweeps(lda_ctx* ctx, int32_t parts, const double* fractions,
                                     int64_t corpus_first_token, int64_t corpus_tokens);
lda_status lda_get_sequential_sweeps(lda_ctx* ctx, int32_t* parts, int64_t* cum_units);
lda_status lda_staleness_schedule(int32_t threads, int32_t* parts, double* fractions);
/* The parts of the sweep in progress (or of the next one) and whether they
 * are sequential (a warm-start sweep) or exchange-overlapped. */
lda_status lda_sweep_parts(lda_ctx* ctx, int32_t* parts, int32_t* sequential);

/* The HIP stream every call of this context is ordered on (hipStream_t;
 * NULL = the context's own stream).  Work already queued on the previous
 * stream is ordered before the new stream's (an event, no host wait). */
lda_status lda_set_stream(lda_ctx* ctx, void* hip_stream);
lda_status lda_get_stream(lda_ctx* ctx, void** hip_stream);
lda_status lda_synchronize(lda_ctx* ctx);

/* Sweep counter (the Philox counter word that keys a sampling pass). */
lda_status lda_get_sweep(lda_ctx* ctx, uint32_t* sweep);
lda_status lda_set_sweep(lda_ctx* ctx, uint32_t sweep);

/* Kp = 64 * C, C the next power of two >= ceil(K/64) (1..64); lane l of a
 * wavefront owns topics [l*C, (l+1)*C). */
int32_t lda_padded_topics(int32_t num_topics);
lda_status lda_get_shape(lda_ctx* ctx, int32_t* K, int32_t* Kp, int32_t* V, int64_t* D,
                         int64_t* N);

/* Copy state out (caller-allocated host buffers; NULL skips an output).
 * z[N]; nw[V*K] row-major (unpadded); nwsum[K]; nd[D*K]; ndsum[D]. */
lda_status lda_get_z(lda_ctx* ctx, int32_t* z);
lda_status lda_set_z(lda_ctx* ctx, const int32_t* z); /* re-seeds counts as pending delta */
lda_status lda_get_counts(lda_ctx* ctx, int32_t* nw, int32_t* nwsum, int32_t* nd,
                          int32_t* ndsum);

/* Replace alpha[K] / beta (host-side hyperparameter optimisation,
 * ParallelTopicModel.optimizeAlpha/optimizeBeta). */
lda_status lda_set_alpha_beta(lda_ctx* ctx, const double* alpha, double beta);

/* ParallelTopicModel.modelLogLikelihood() over this shard's documents:
 * doc_part = sum_d [sum_k logG(a_k+n_dk)-logG(a_k)] - logG(A+n_d) + logG(A)
 * (fp64, Dirichlet.logGammaStirling); word_part = the nw/nwsum terms (global,
 * identical on every rank).  Total = sum over ranks of doc_part + word_part. */
lda_status lda_log_likelihood_parts(lda_ctx* ctx, double* doc_part, double* word_part);
lda_status lda_log_likelihood(lda_ctx* ctx, double* out); /* doc_part + word_part */
/* The same without waiting: the kernels and the copy of their partial sums
 * are enqueued on the context's stream, and the result is collected later
 * (ParallelTopicModel.estimate()'s "LL/token" every 10 sweeps no longer
 * stops the sweeps).  At most 16 results in flight: a 17th enqueue waits
 * for the oldest, whose ticket then no longer collects (LDA_ERR_STATE). */
lda_status lda_log_likelihood_enqueue(lda_ctx* ctx, int64_t* ticket);
lda_status lda_log_likelihood_collect(lda_ctx* ctx, int64_t ticket, double* doc_part, double* word_part);

/* TopicInferencer.getSampledDistribution(instance, numIterations, thinning,
 * burnIn) [src/cmu_ron/TrainAndPredict.java:144, src/cmu/TrainAndPredict.java:114]
 * batched over Dh held-out documents against the frozen model; the arguments
 * are in Mallet's order.  Word ids must be < V (out-of-vocabulary tokens are
 * removed by the caller); tokens whose type has no training tokens (an empty
 * typeTopicCounts row) are skipped, as Mallet's inferencer skips them.
 * theta[Dh*K] (fp64, rows sum to 1). */
lda_status lda_infer(lda_ctx* ctx, int64_t Dh, const int64_t* doc_off, const int32_t* words,
                     int32_t num_iterations, int32_t thinning, int32_t burn_in, uint64_t seed,
                     double* theta);

/* Mallet-layout adapter: typeTopicCounts as packed (count << topic_bits) |
 * topic rows sorted descending, rows[row_off[w] .. row_off[w+1]) with
 * row_off[V+1]; row length = min(K, typeTotal[w]) exactly as Mallet allocates
 * it, trailing cells 0.  Pass rows = NULL to get row_off / total / topic_bits
 * only. */
lda_status lda_to_mallet_packed(lda_ctx* ctx, int32_t* rows, int64_t* row_off,
                                int32_t* topic_bits);

/* ---- hyperparameter optimisation ----------------------
 * Mallet 2.0.7 ParallelTopicModel.optimizeAlpha / optimizeBeta, enabled by
 * setOptimizeInterval(20) [src/cmu_ron/TrainAndPredict.java:163,
 * src/cmu/TrainAndPredict.java:261].  The GPU builds the integer statistics;
 * the fp64 fixed-point updates run on the host. */

/* Longest document of this shard (sizes the histograms below). */
lda_status lda_max_doc_length(lda_ctx* ctx, int32_t* max_len);
/* WorkerRunnable's alpha statistics from the current z of this shard, ADDED
 * into caller buffers (accumulate over the sampled sweeps, sum across ranks):
 * doc_len_counts[max_len+1]: documents of each length (docLengthCounts);
 * topic_doc_counts[K*(max_len+1)], row k: documents in which topic k has
 * each count > 0 (topicDocCounts).  max_len >= lda_max_doc_length. */
lda_status lda_doc_topic_histograms(lda_ctx* ctx, int32_t max_len, int32_t* doc_len_counts,
                                    int32_t* topic_doc_counts);
/* The same statistics summed on the device over several sweeps without a
 * host round trip: _accumulate adds the current z's histograms into the
 * context's own buffer, _take ADDS the sum into the caller's buffers and
 * zeroes it, _clear zeroes it.  max_len must stay the same between takes. */
lda_status lda_doc_topic_histograms_accumulate(lda_ctx* ctx, int32_t max_len);
lda_status lda_doc_topic_histograms_take(lda_ctx* ctx, int32_t max_len, int32_t* doc_len_counts,
                                         int32_t* topic_doc_counts);
lda_status lda_doc_topic_histograms_clear(lda_ctx* ctx);
/* optimizeBeta's countHistogram, ADDED into count_hist[max_count+1]: cells
 * (w, k) of the global nw holding each count c > 0 (identical on every rank:
 * do not sum it across ranks).  LDA_ERR_INVALID_ARG if a cell exceeds
 * max_count (the largest word total bounds every cell). */
lda_status lda_count_histogram(lda_ctx* ctx, int64_t max_count, int32_t* count_hist);
/* One optimisation step's statistics with a single wait on the stream (the
 * three calls above and lda_get_counts' nwsum each wait on their own): the
 * accumulated document histograms ADDED and zeroed as _take (when
 * doc_len_counts / topic_doc_counts are non-null), the count histogram ADDED
 * (count_hist non-null), nwsum[K] copied (non-null).  Each output is optional.
 * Replaces the per-statistic round trips of ParallelTopicModel.estimate()'s
 * optimizeAlpha / optimizeBeta (ParallelTopicModel.java 2.0.7). */
lda_status lda_hyper_statistics(lda_ctx* ctx, int32_t max_len, int32_t* doc_len_counts,
                                int32_t* topic_doc_counts, int64_t max_count, int32_t* count_hist,
                                int32_t* nwsum);

/* Dirichlet.learnParameters(params, observations, observationLengths, shape,
 * scale, iterations): Minka's fixed point with a Gamma(shape, scale) prior;
 * params[K] updated in place, params_sum = their new sum.  Host-only. */
lda_status lda_learn_parameters(double* params, int32_t K, const int32_t* observations,
                                const int32_t* observation_lengths, int32_t max_len, double shape,
                                double scale, int32_t iterations, double* params_sum);
/* Dirichlet.learnSymmetricConcentration(countHistogram, observationLengths,
 * numDimensions, currentValue): 200 fixed-point steps for a symmetric
 * Dirichlet's total concentration.  count_hist[max_count+1]; the observation
 * length histogram is given sparsely as ascending (lengths[j], length_counts[j])
 * pairs (topic sizes reach ~1e9 at C4).  Host-only. */
lda_status lda_learn_symmetric_concentration(const int32_t* count_hist, int64_t max_count,
                                             const int64_t* lengths, const int32_t* length_counts,
                                             int64_t n_lengths, int32_t num_dims, double current,
                                             double* out);
/* Dirichlet.digamma (the series the estimators use).  Host-only. */
double lda_digamma(double z);

/* Token-weighted mean number of nonzero topics in a token's word row of the
 * current (global) snapshot: sum_w n_w * nnz(nw[w]) / sum_w n_w.  The sparse
 * samplers read 4 bytes per such entry (SURVEY.md §8d's B_sparse). */
lda_status lda_row_stats(lda_ctx* ctx, double* mean_row_nnz);

/* Kernel-level timing of the last lda_sample (ms, HIP events on the
 * context's stream). */
lda_status lda_last_sample_ms(lda_ctx* ctx, float* ms);
/* Kernel durations (ms, oldest first) of the last n = min(max, launches, 256)
 * lda_sample calls: bench.py reads the launches of its timed region. */
lda_status lda_sample_times(lda_ctx* ctx, int32_t max, float* ms, int32_t* n);
/* The same for the recount kernel that follows each sampler launch in the
 * recount mode (0 ms in the delta mode). */
lda_status lda_recount_times(lda_ctx* ctx, int32_t max, float* ms, int32_t* n);

/* Diagnostics: the sampler's own uniform draws on the current device.
 * out[i] = word 0 of Philox4x32-10 with counter {gtok[i] lo, gtok[i] hi, c2,
 * c3} and key {seed lo, seed hi} -- the x0 every kernel draws (c2 = sweep,
 * c3 = stream: 0 sample, 1 init, 2 inference).  Used to pin the device RNG
 * against rocRAND's philox4x32_10 (tests/native/philox_vs_rocrand.hip). */
lda_status lda_philox_draws(uint64_t seed, uint32_t c2, uint32_t c3, const int64_t* gtok, int64_t n,
                            uint32_t* out);

const char* lda_last_error(void);
/* Test hook: the nth host allocation of a caller-sized buffer on this thread
 * (counted from this call; 0 = off) fails with std::bad_alloc, which the
 * entry point reports as LDA_ERR_OUT_OF_MEMORY (tests/test_abi_guard*.py). */
void lda_debug_fail_host_alloc(int32_t nth);
/* "lda_mi355x <version> (gfx950; ABI <n>)".  ABI history: 2 -- lda_infer's
 * last three ints became (num_iterations, thinning, burn_in), Mallet's
 * getSampledDistribution order (was (n_iter, burn_in, thin)); 3 -- the dense
 * samplers' exchange buffer holds recounted counts (lda_count_update_mode),
 * lda_recount_times, lda_set_exchange_parts' reserve_cus < 0 = default; 4 --
 * lda_hyper_statistics, lda_set_alpha_beta returns without waiting for the
 * stream (its upload is asynchronous); 5 -- warm-start parts are interleaved
 * segments of the corpus (LDA_WARM_BLOCKS), lda_warm_part_tokens; 6 -- the
 * large-K sampler's draw (C >= 32: exact fixed-point doc part, own-entry
 * accept / re-draw), sequential sweeps recount under LDA_COUNT_RECOUNT,
 * lda_exchange_unpack_lists, lda_counts_checksum; 7 -- lda_set_exchange_cells
 * (four 8-bit cells per packed word). */
#define LDA_ABI_VERSION 7
const char* lda_version(void);
int32_t lda_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* LDA_MI355X_H */
