/*
 * lda_topic_model.h — C ABI of the native host mirror of Mallet 2.0.7's
 * ParallelTopicModel / TopicInferencer, built on the sampler ABI in
 * lda_mi355x.h (liblda_topic_model.so, C++: ldagibbssampling_amd/host/).
 *
 * The reference drives Mallet through exactly this surface
 * (src/cmu_ron/TrainAndPredict.java:159-177, 230-234, 108-156;
 * src/cmu/TrainAndPredict.java:93-114, 258-274, 436):
 *   new ParallelTopicModel(K, alphaSum, beta)     -> ldatm_create
 *   addInstances(InstanceList)                    -> ldatm_set_alphabet + ldatm_add_instances
 *   setOptimizeInterval / setNumThreads /
 *   setNumIterations / setTopicDisplay            -> ldatm_set_*
 *   estimate()                                    -> ldatm_estimate
 *   modelLogLikelihood()                          -> ldatm_model_log_likelihood
 *   getTopicProbabilities(topicSequence)          -> ldatm_get_topic_probabilities
 *   printDocumentTopics(File)                     -> ldatm_print_document_topics
 *   printTopWords(File, n, newLines)              -> ldatm_print_top_words
 *   getInferencer().getSampledDistribution(...)   -> ldatm_infer
 * Word ids index the model's alphabet (Mallet's Alphabet: insertion order).
 * Errors: lda_status codes of lda_mi355x.h, message in ldatm_last_error().
 */
#ifndef LDA_TOPIC_MODEL_H
#define LDA_TOPIC_MODEL_H

#include <stddef.h>
#include <stdint.h>

#include "lda_mi355x.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ldatm ldatm;

/* ParallelTopicModel(numberOfTopics, alphaSum, beta): alpha_k = alphaSum/K. */
lda_status ldatm_create(ldatm** out, int32_t num_topics, double alpha_sum, double beta);
void ldatm_destroy(ldatm* m);

/* The InstanceList's data alphabet (UTF-8 words, index = word id).  words may
 * be NULL: ids only (top-words output then prints the ids).  Growing the
 * alphabet between addInstances calls is allowed (updateModel). */
lda_status ldatm_set_alphabet(ldatm* m, int32_t num_types, const char* const* words);
/* addInstances: D documents (doc_off[D+1], words[...] word ids < num_types of
 * the alphabet), sources[D] (Instance.getSource(), NULL or NULL entries ->
 * "null-source").  New documents get random topics (Philox, keyed by the
 * global token index); documents already added keep theirs. */
lda_status ldatm_add_instances(ldatm* m, int64_t D, const int64_t* doc_off, const int32_t* words,
                               const char* const* sources);

lda_status ldatm_set_num_iterations(ldatm* m, int32_t n);      /* setNumIterations   */
lda_status ldatm_set_optimize_interval(ldatm* m, int32_t n);   /* setOptimizeInterval */
lda_status ldatm_set_burnin_period(ldatm* m, int32_t n);       /* setBurninPeriod (200) */
lda_status ldatm_set_save_sample_interval(ldatm* m, int32_t n);/* saveSampleInterval (10) */
lda_status ldatm_set_symmetric_alpha(ldatm* m, int32_t on);    /* setSymmetricAlpha  */
lda_status ldatm_set_topic_display(ldatm* m, int32_t interval, int32_t n); /* setTopicDisplay */
lda_status ldatm_set_random_seed(ldatm* m, int64_t seed);      /* setRandomSeed      */
/* setNumThreads: Mallet's document blocks.  Here a block is a GPU shard:
 * ldatm_plan_shards(n, visible devices, corpus) GPUs -- at most n and the
 * devices, and ONE when the sweep is too short to pay for the exchange (the
 * reference's own ~16k-token corpus with setNumThreads(4)) -- with an RCCL
 * all-reduce of the exchange buffer between them.  Results do not depend on
 * it (integer sums, global Philox counters). */
lda_status ldatm_set_num_threads(ldatm* m, int32_t n);
/* The shard plan of setNumThreads (host-only): min(num_threads, num_devices,
 * num_docs) shards, reduced while (1 - 1/G) of the estimated sweep time
 * (num_tokens x (2 Kp + 16) bytes at 5 TB/s) does not exceed the estimated
 * ring all-reduce of 4 (V Kp + Kp) bytes (100 GB/s per link + 100 us). */
int32_t ldatm_plan_shards(int32_t num_threads, int32_t num_devices, int64_t num_tokens,
                          int32_t num_types, int32_t num_topics, int64_t num_docs);
/* Explicit shard placement: n shards, shard g on HIP device devices[g]
 * (n = 0: back to setNumThreads' plan).  Shards on distinct devices exchange
 * through RCCL; shards that ALL share one device exchange through a
 * device-side sum with the same streams, events and apply ordering (the
 * multi-shard path on a one-GPU box).  Other mixes: LDA_ERR_UNSUPPORTED. */
lda_status ldatm_set_devices(ldatm* m, int32_t n, const int32_t* devices);
/* Shards the next estimate() runs on (creates them if needed). */
lda_status ldatm_num_shards(ldatm* m, int32_t* shards);
/* The shards' compact exchange (lda_exchange_pack; creates the shards if
 * needed): cells per packed word (lda_set_exchange_cells: 4 for K > 1024 up
 * to 64 shards, else 2; 0 when the shards do not exchange packed words --
 * one shard, or shards on one device without LDA_LOCAL_COMPACT=1), whether
 * the escape lists travel at their used length (1, the default: the counts
 * are read on the host behind each pack, overlapping the packed words'
 * all-reduce) or whole (0, LDA_ESCAPE_LISTS=capacity), the largest per-shard
 * escape count gathered so far and the number of count reads.  Any pointer
 * may be NULL. */
lda_status ldatm_exchange_info(ldatm* m, int32_t* cells_per_word, int32_t* used_lists, int32_t* escapes_max,
                               int64_t* list_exchanges);
/* LDA_SAMPLER_* (default: DENSE for K <= 1024, SPARSE above) */
lda_status ldatm_set_sampler(ldatm* m, int32_t sampler);
/* With more than one GPU shard: cut every sweep into `parts` parts
 * (1..LDA_MAX_EXCHANGE_PARTS) whose all-reduces overlap the next part's
 * sampling (lda_set_exchange_parts).  No effect on one GPU or on results. */
lda_status ldatm_set_exchange_parts(ldatm* m, int32_t parts);
/* Warm start (lda_set_warm_start): sweeps 0 .. sweeps-1 of the model's sweep
 * counter run in `parts` sequential parts, so that the early sweeps see part
 * of their own changes as Mallet's worker threads do.  Default 4 parts x 50
 * sweeps (held-out perplexity at K = 20 over 48 seeds: 10 / 48 seeds in a
 * worse local optimum instead of 18 / 48; cpu_mallet 16 / 48).
 * (1, 0) turns it off.  Carried by checkpoints and by the sweep counter. */
lda_status ldatm_set_warm_start(ldatm* m, int32_t parts, int32_t sweeps);
/* Sweeps past the warm start show each token the share of the sweep's other
 * changes that Mallet's T worker threads would (lda_set_sequential_sweeps /
 * lda_staleness_schedule): threads = 0 (the default) takes T
 * from ldatm_set_num_threads (the reference's setNumThreads(4)), threads > 0
 * sets T, threads < 0 runs plain snapshot sweeps.  Without it the learned
 * hyperparameters drift from Mallet's at the reference's settings (beta
 * ~9% high, alphaSum ~4% low) and K = 500 traps more chains.  Carried by
 * checkpoints (files before format v3 continue with snapshot sweeps). */
lda_status ldatm_set_staleness_threads(ldatm* m, int32_t threads);
/* State a Java-side ParallelTopicModel already holds, for GpuParallelTopicModel
 * (integration/): the topics Mallet's own addInstances drew (z[n], n = every
 * token of the model), alpha[K] / alphaSum / beta after an earlier optimisation,
 * and the Philox sweep counter, which must continue across estimate() calls
 * (updateModel, src/cmu_ron/TrainAndPredict.java:173-177) so that a second
 * estimate() does not replay the first one's uniforms. */
lda_status ldatm_set_topics(ldatm* m, int64_t n, const int32_t* z);
lda_status ldatm_set_hyper(ldatm* m, const double* alpha, double alpha_sum, double beta);
lda_status ldatm_get_sweep(ldatm* m, uint32_t* sweep);
lda_status ldatm_set_sweep(ldatm* m, uint32_t sweep);
/* printLogLikelihood / logging: 0 = silent, 1 = Mallet's INFO lines on stderr */
lda_status ldatm_set_verbosity(ldatm* m, int32_t level);
lda_status ldatm_set_print_log_likelihood(ldatm* m, int32_t on);

/* estimate(): numIterations sweeps; statistics every saveSampleInterval and
 * optimizeAlpha/optimizeBeta every optimizeInterval sweeps after the burn-in;
 * LL/token every 10 sweeps (kept in the trace below). */
lda_status ldatm_estimate(ldatm* m);
/* (iteration, LL/token) pairs of the last estimate(): n = number available;
 * copies min(cap, n). */
lda_status ldatm_get_ll_trace(ldatm* m, int32_t* iterations, double* ll_per_token, int32_t cap,
                              int32_t* n);

lda_status ldatm_model_log_likelihood(ldatm* m, double* out);
lda_status ldatm_get_shape(ldatm* m, int32_t* K, int32_t* V, int64_t* D, int64_t* N);
lda_status ldatm_get_hyper(ldatm* m, double* alpha /*[K]*/, double* alpha_sum, double* beta);
lda_status ldatm_get_z(ldatm* m, int32_t* z /*[N]*/);
lda_status ldatm_get_counts(ldatm* m, int32_t* nw /*[V*K] or NULL*/, int32_t* nwsum /*[K]*/);
/* getTopicProbabilities(doc): (n_dk + alpha_k) / sum_k (n_dk + alpha_k). */
lda_status ldatm_get_topic_probabilities(ldatm* m, int64_t doc, double* out /*[K]*/);

/* printDocumentTopics(File) (threshold 0, max -1 = all) and its text:
 * "#doc source topic proportion ...", then per document
 * "<doc> <source|null-source> <topic> <weight> ... \n" (weights descending,
 * Java Double.toString).  printTopWords(File, numWords, usingNewLines):
 * displayTopWords text ("<topic>\t<alpha>\t<word> <word> ...\n").
 * The *_text variants write into buf (cap bytes incl. NUL) and report the
 * full length in *len (call with buf = NULL to size it). */
lda_status ldatm_print_document_topics(ldatm* m, const char* path, double threshold, int32_t max);
lda_status ldatm_document_topics_text(ldatm* m, double threshold, int32_t max, char* buf,
                                      size_t cap, size_t* len);
lda_status ldatm_print_top_words(ldatm* m, const char* path, int32_t num_words,
                                 int32_t using_new_lines);
lda_status ldatm_top_words_text(ldatm* m, int32_t num_words, int32_t using_new_lines, char* buf,
                                size_t cap, size_t* len);

/* Checkpoint / resume: the reference's save()/load() of its model
 * (src/cmu_ron/TrainAndPredict.java:179-200) as a native binary file holding
 * every field needed to continue bit for bit (documents, alphabet, sources,
 * topics, alpha/beta, options, pending optimisation statistics and the
 * Philox sweep counter).  ldatm_load creates a new model. */
lda_status ldatm_save(ldatm* m, const char* path);
lda_status ldatm_load(ldatm** out, const char* path);

/* getInferencer().getSampledDistribution(instance, numIterations, thinning,
 * burnIn) [src/cmu_ron/TrainAndPredict.java:144], batched over Dh documents
 * (word ids of the model alphabet; ids >= V are dropped like Mallet's
 * unknown-type tokens).  theta[Dh*K]. */
lda_status ldatm_infer(ldatm* m, int64_t Dh, const int64_t* doc_off, const int32_t* words,
                       int32_t num_iterations, int32_t thinning, int32_t burn_in, uint64_t seed,
                       double* theta);

/* The number renderings of Mallet's text outputs (host-only): style 0 =
 * Double.toString (printDocumentTopics weights), 1 = NumberFormat with at
 * most 5 fraction digits (printTopWords alpha, LL/token log). */
lda_status ldatm_format_double(double x, int32_t style, char* buf, size_t cap);

const char* ldatm_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* LDA_TOPIC_MODEL_H */
