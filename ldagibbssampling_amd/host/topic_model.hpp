// topic_model.hpp — native host mirror of Mallet 2.0.7's ParallelTopicModel
// (cc.mallet.topics, not vendored; pom.xml:107-111) over the sampler C ABI.
//
// What the reference calls (src/cmu_ron/TrainAndPredict.java:159-177,
// src/cmu/TrainAndPredict.java:258-274) keeps its name and meaning here; the
// per-token sampling inside estimate() is the GPU (lda_sample / lda_apply on
// one context per GPU shard, RCCL all-reduce of the int32 delta between them).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/lda_mi355x.h"

namespace lda_host {

struct Error {
  lda_status status;
  std::string message;
};

class ShardGroup;  // GPU shards + their all-reduce (topic_model.cpp)

// GPU shards for setNumThreads(num_threads) over this corpus (ldatm_plan_shards)
int32_t plan_shards(int32_t num_threads, int32_t num_devices, int64_t num_tokens, int32_t num_types,
                    int32_t num_topics, int64_t num_docs);

class ParallelTopicModel {
 public:
  ParallelTopicModel(int32_t num_topics, double alpha_sum, double beta);
  ~ParallelTopicModel();
  ParallelTopicModel(const ParallelTopicModel&) = delete;
  ParallelTopicModel& operator=(const ParallelTopicModel&) = delete;

  // ---- data (addInstances) -------------------------------------------
  void setAlphabet(std::vector<std::string> words, int32_t num_types);
  void addInstances(int64_t D, const int64_t* doc_off, const int32_t* words,
                    const char* const* sources);

  // ---- options -------------------------------------------------------
  void setNumIterations(int32_t n) { num_iterations_ = n; }
  void setOptimizeInterval(int32_t n) { optimize_interval_ = n; }
  void setBurninPeriod(int32_t n) { burnin_period_ = n; }
  void setSaveSampleInterval(int32_t n) { save_sample_interval_ = n; }
  void setSymmetricAlpha(bool on) { symmetric_alpha_ = on; }
  void setTopicDisplay(int32_t interval, int32_t n) {
    show_topics_interval_ = interval;
    words_per_topic_ = n;
  }
  void setRandomSeed(int64_t seed);
  void setNumThreads(int32_t n);
  void setSampler(int32_t sampler);
  // split sweeps across GPU shards: each shard's sweep in `parts` parts, part
  // i's all-reduce overlapping part i+1's sampling (1 = one exchange per sweep)
  void setExchangeParts(int32_t parts);
  // explicit shard placement: shard g on devices[g] (n shards; n = 0 returns
  // to setNumThreads' plan).  Shards that share one device exchange through a
  // device-side sum instead of RCCL (the multi-shard path on one GPU).
  void setDevices(const int32_t* devices, int32_t n);
  // warm start (lda_set_warm_start): sweeps 0..sweeps-1 in `parts` sequential
  // parts; the default 4 x 50 (held-out perplexity at K = 20)
  void setWarmStart(int32_t parts, int32_t sweeps);
  // sweeps past the warm start emulate the staleness of Mallet's T worker
  // threads (lda_staleness_schedule): T = 0 -> numThreads (the default),
  // T < 0 -> plain snapshot sweeps
  void setStalenessThreads(int32_t threads);
  int32_t numShards();
  // the shards' compact exchange: cells per packed word (0: not compact),
  // escape lists at their used length (1) or whole, the largest per-shard
  // escape count gathered and the count reads so far (ldatm_exchange_info)
  void exchangeInfo(int32_t* cells, int32_t* used_lists, int32_t* escapes_max, int64_t* list_exchanges);
  void setVerbosity(int32_t v) { verbosity_ = v; }
  // state a Java-side ParallelTopicModel already holds (GpuParallelTopicModel:
  // Mallet's own addInstances topics, alpha/beta optimised in an earlier
  // estimate(), the Philox sweep counter of the previous estimate())
  void setTopics(const int32_t* z, int64_t n);
  void setHyper(const double* alpha, double alpha_sum, double beta);
  uint32_t sweep();
  void setSweep(uint32_t s);
  void setPrintLogLikelihood(bool on) { print_log_likelihood_ = on; }

  // ---- training ------------------------------------------------------
  void estimate();
  const std::vector<std::pair<int32_t, double>>& llTrace() const { return ll_trace_; }
  double modelLogLikelihood();

  // ---- state ---------------------------------------------------------
  int32_t numTopics() const { return K_; }
  int32_t numTypes() const { return V_; }
  int64_t numDocs() const { return (int64_t)doc_off_.size() - 1; }
  int64_t numTokens() const { return doc_off_.back(); }
  const std::vector<double>& alpha() const { return alpha_; }
  double alphaSum() const { return alpha_sum_; }
  double beta() const { return beta_; }
  std::vector<int32_t> topics();                      // z of every token
  void counts(int32_t* nw, int32_t* nwsum);           // nw[V*K] (nullable), nwsum[K]
  std::vector<double> getTopicProbabilities(int64_t doc);

  // ---- outputs -------------------------------------------------------
  std::string documentTopics(double threshold, int32_t max);
  std::string displayTopWords(int32_t num_words, bool using_new_lines);

  // ---- checkpoint / resume (the reference's save()/load(),
  //      src/cmu_ron/TrainAndPredict.java:179-200, as a native format) ----
  void save(const std::string& path);
  static std::unique_ptr<ParallelTopicModel> load(const std::string& path);

  // ---- inference (TopicInferencer.getSampledDistribution, batched) ---
  void infer(int64_t Dh, const int64_t* doc_off, const int32_t* words, int32_t num_iterations,
             int32_t thinning, int32_t burn_in, uint64_t seed, double* theta);

 private:
  void ensureShards();
  void markDirty();
  void optimizeAlpha();
  // count histogram (max_word_total_ + 1 cells) and nwsum, fetched with the
  // alpha statistics in one lda_hyper_statistics call
  void optimizeBeta(const std::vector<int32_t>& count_hist, const std::vector<int32_t>& nwsum);
  void log(const std::string& line) const;

  int32_t K_;
  double alpha_sum_, beta_;
  std::vector<double> alpha_;
  int32_t V_ = 0;
  std::vector<std::string> alphabet_;
  std::vector<int64_t> doc_off_{0};
  std::vector<int32_t> words_;
  std::vector<std::string> sources_;
  std::vector<uint8_t> has_source_;
  std::vector<int32_t> z_cache_;  // z of the shards, valid when !z_dirty_
  bool z_dirty_ = true;

  int32_t num_iterations_ = 1000, optimize_interval_ = 0, burnin_period_ = 200;
  int32_t save_sample_interval_ = 10, show_topics_interval_ = 50, words_per_topic_ = 7;
  bool symmetric_alpha_ = false, print_log_likelihood_ = true;
  uint64_t seed_ = 0;
  int32_t num_threads_ = 1, sampler_ = LDA_SAMPLER_DENSE, verbosity_ = 0, exchange_parts_ = 1;
  // shards on distinct GPUs exchange packed words (lda_exchange_pack);
  // LDA_EXCHANGE_INT32=1 in the environment sends the int32 buffers (A/B)
  bool compact_exchange_ = true;
  int32_t warm_parts_ = 4, warm_sweeps_ = 50;
  int32_t staleness_threads_ = 0;
  void applySweepSchedule();

  std::vector<int32_t> devices_;  // setDevices (empty: plan_shards)
  std::unique_ptr<ShardGroup> shards_;
  bool shards_dirty_ = true;
  int32_t max_doc_len_ = -1;
  int64_t max_word_total_ = 0;  // largest word frequency (countHistogram bound), set with the shards
  uint32_t sweep_ = 0;  // Philox sweep counter carried across re-sharding
  std::vector<int32_t> doc_len_counts_, topic_doc_counts_;  // alpha statistics
  std::vector<std::pair<int32_t, double>> ll_trace_;
};

}  // namespace lda_host
