// topic_model.cpp — ParallelTopicModel host mirror (see topic_model.hpp) and
// the C ABI of include/lda_topic_model.h.
//
// Mallet 2.0.7 behaviour restated here (cc.mallet.topics.ParallelTopicModel,
// not vendored; call sites src/cmu_ron/TrainAndPredict.java:159-177):
//  * addInstances: new documents get random topics, earlier ones keep theirs;
//    counts are rebuilt from every document.
//  * estimate(): for iteration = 1..numIterations: topic display every
//    showTopicsInterval; one parallel sweep (AD-LDA: every shard samples
//    against the same nw snapshot, then the deltas are summed); alpha
//    statistics on sweeps with iteration > burninPeriod and
//    iteration % saveSampleInterval == 0; optimizeAlpha + optimizeBeta when
//    iteration > burninPeriod and iteration % optimizeInterval == 0;
//    "<iteration> LL/token: x" every 10 iterations.
//  * optimizeAlpha: Dirichlet.learnParameters(alpha, topicDocCounts,
//    docLengthCounts, 1.001, 1.0, 1), or learnSymmetricConcentration over the
//    pooled histogram when usingSymmetricAlpha; histograms then cleared.
//  * optimizeBeta: learnSymmetricConcentration(countHistogram,
//    topicSizeHistogram, numTypes, betaSum); beta = betaSum / numTypes.
#include "topic_model.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdlib>
#include <climits>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <numeric>
#include <sstream>

#include "../../include/lda_topic_model.h"
#include "java_format.hpp"

namespace lda_host {

namespace {

[[noreturn]] void raise(lda_status s, const std::string& msg) { throw Error{s, msg}; }

void check(lda_status s, const char* where) {
  if (s != LDA_OK) {
    const char* m = lda_last_error();
    raise(s, std::string(where) + ": " + (m ? m : ""));
  }
}

// dst[i] += src[i]: the in-process sum of shard buffers that share one device
// (ShardGroup's local exchange; RCCL refuses two ranks on one GPU)
__global__ void k_sum_into(int4* __restrict__ dst, const int4* __restrict__ src, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    const int4 b = src[i];
    if (b.x | b.y | b.z | b.w) {
      int4 a = dst[i];
      a.x += b.x;
      a.y += b.y;
      a.z += b.z;
      a.w += b.w;
      dst[i] = a;
    }
  }
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) raise(e == hipErrorOutOfMemory ? LDA_ERR_OUT_OF_MEMORY : LDA_ERR_DEVICE,
                             std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// How many GPU shards setNumThreads(n) becomes (ldatm_plan_shards): at most
// n, the visible devices and the documents, and one when splitting the
// sweep saves less than the exchange costs.  Per sweep, the sampler moves
// ~(2 Kp + 16) bytes per token (the 16-bit row + stream; the sparse kernels
// read fewer bytes at a lower rate) at ~5 TB/s, the exchange is a ring
// all-reduce of 4 (V Kp + Kp) bytes at ~100 GB/s per link plus ~100 us of
// latency; G shards save (1 - 1/G) of the sweep.  The reference's own corpus
// (C1: ~16k tokens, K = 500, V ~ 5000) with setNumThreads(4) gets one GPU: its
// ~40 us sweep is far below a 10 MB all-reduce.
int32_t plan_shards(int32_t num_threads, int32_t num_devices, int64_t num_tokens, int32_t num_types,
                    int32_t num_topics, int64_t num_docs) {
  const int64_t g = std::max<int64_t>(1, std::min<int64_t>({(int64_t)num_threads, (int64_t)num_devices,
                                                            std::max<int64_t>(num_docs, 1)}));
  if (g < 2) return 1;
  const double kp = (double)lda_padded_topics(num_topics);
  const double sweep_s = (double)num_tokens * (2.0 * kp + 16.0) / 5e12;
  const double exch_s = 2.0 * 4.0 * ((double)num_types * kp + kp) / 1e11 + 1e-4;
  for (int64_t k = g; k >= 2; --k)
    if (sweep_s * (1.0 - 1.0 / (double)k) > exch_s) return (int32_t)k;
  return 1;
}

// ----------------------------------------------------------------- shards
// One lda_ctx per GPU over a contiguous, token-balanced document range; the
// delta buffers are summed in place with one RCCL all-reduce per sweep
// (ncclCommInitAll over the shards' devices, grouped calls from this thread).
//
// Split sweeps (setExchangeParts, lda_set_exchange_parts): every shard samples
// its documents in P parts with one delta buffer each; part i's all-reduce is
// issued on a per-shard collective stream that waits only for part i, so it
// runs while part i+1 samples, and the shards' streams wait for the last sum
// before the apply.  Same sweep bit for bit (integer sums, fixed snapshot).
//
// Shards on distinct devices exchange through RCCL.  Shards that share one
// device (ParallelTopicModel::setDevices, e.g. {0, 0, 0}: the multi-shard
// path exercised on a one-GPU box) exchange through a device-side sum
// instead -- shard 0's stream adds every other buffer into its own and copies
// the sum back -- with the same events, streams and apply ordering.
class ShardGroup {
 public:
  std::vector<lda_ctx*> ctx;
  std::vector<int> dev;            // shard g runs on device dev[g]
  std::vector<int64_t> doc_begin;  // shard g owns documents [doc_begin[g], doc_begin[g+1])
  bool local_sum = false;          // every shard on one device: no RCCL
  std::vector<ncclComm_t> comms;
  std::vector<hipStream_t> comm_streams;  // per shard, split sweeps only
  std::vector<hipEvent_t> events;
  std::vector<hipEvent_t> sum_events;     // local_sum: per shard "sampled" / shard 0 "summed"
  int parts = 1;
  // RCCL exchange in the compact form (lda_exchange_pack): the largest
  // shard's tokens (sizes the escape lists), the packed words and escape
  // list of every shard per part, and per shard and part the gathered lists
  // of all shards [G x escape_count]
  int64_t max_tokens = 0;
  bool compact = true;
  // shards on one device exchange the compact form through device-side
  // stand-ins for the collectives (sum of the packed words, copies of the
  // escape lists): the pack / unpack ordering of the multi-GPU path, run on a
  // one-GPU box (LDA_LOCAL_COMPACT=1; tests/test_topic_model_gpu.py)
  bool local_compact = false;
  size_t packed_count = 0, escape_count = 0;
  std::vector<std::vector<void*>> packed, escapes;        // [part][shard]
  std::vector<std::vector<int32_t*>> escapes_all;         // [part][shard], device buffers
  // escape lists at their used length (round 6, the torch path's default
  // since round 5): every shard's count is copied to pinned host memory right
  // behind its pack, the packed words' all-reduce is issued, and only then
  // does the host read the counts (the copies, not the sum: the read overlaps
  // that collective) and all-gather 1 + 3 m int32 per shard, m the largest
  // count; nothing when m = 0.  false: the whole fixed-capacity lists, no
  // read (LDA_ESCAPE_LISTS=capacity).
  bool used_lists = true;
  int32_t cells = 2;                                      // lda_set_exchange_cells
  int32_t* host_counts = nullptr;                         // pinned [LDA_MAX_EXCHANGE_PARTS][G]
  std::vector<std::vector<hipEvent_t>> count_events;      // [part][shard]: count copied
  std::vector<size_t> gathered_cap;                       // [part]: escapes_all holds G x this
  std::vector<int32_t> part_m;                            // [part]: the m of the pending exchange
  int32_t m_max = 0;                                      // largest m gathered (ldatm_exchange_info)
  int64_t list_exchanges = 0;                             // count reads so far

  ~ShardGroup() {
    for (auto c : comms) ncclCommDestroy(c);
    for (size_t g = 0; g < comm_streams.size(); ++g) {
      (void)hipSetDevice(dev[g]);
      (void)hipEventDestroy(events[g]);
      (void)hipStreamDestroy(comm_streams[g]);
    }
    for (size_t g = 0; g < sum_events.size(); ++g) {
      (void)hipSetDevice(dev[g]);
      (void)hipEventDestroy(sum_events[g]);
    }
    for (auto& v : escapes_all)
      for (size_t g = 0; g < v.size(); ++g)
        if (v[g]) {
          (void)hipSetDevice(dev[g]);
          (void)hipFree(v[g]);
        }
    for (auto& v : count_events)
      for (size_t g = 0; g < v.size(); ++g) {
        (void)hipSetDevice(dev[g]);
        (void)hipEventDestroy(v[g]);
      }
    if (host_counts) (void)hipHostFree(host_counts);
    for (auto c : ctx) lda_destroy(c);
  }

  void init_exchange() {
    const size_t G = ctx.size();
    if (G < 2) return;
    local_sum = std::all_of(dev.begin(), dev.end(), [&](int d) { return d == dev[0]; });
    if (local_sum) {
      sum_events.resize(G);
      hip_check(hipSetDevice(dev[0]), "hipSetDevice");
      for (size_t g = 0; g < G; ++g)
        hip_check(hipEventCreateWithFlags(&sum_events[g], hipEventDisableTiming), "hipEventCreate");
      return;
    }
    std::vector<int> sorted = dev;
    std::sort(sorted.begin(), sorted.end());
    if (std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end())
      raise(LDA_ERR_UNSUPPORTED, "shards share a device with others on different devices: place all on "
                                 "one device or each on its own");
    comms.resize(G);
    const ncclResult_t r = ncclCommInitAll(comms.data(), (int)G, dev.data());
    if (r != ncclSuccess) {
      comms.clear();
      raise(LDA_ERR_DEVICE, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    }
  }

  // local_sum: buffer 0 += buffer g, then every buffer = buffer 0, on
  // streams[0] once every shard's streams[g] has reached this point; the
  // other streams then wait for the sum
  void local_reduce(const std::vector<void*>& ptr, size_t count, const std::vector<hipStream_t>& streams) {
    const size_t G = ctx.size();
    hip_check(hipSetDevice(dev[0]), "hipSetDevice");
    for (size_t g = 1; g < G; ++g) {
      hip_check(hipEventRecord(sum_events[g], streams[g]), "hipEventRecord");
      hip_check(hipStreamWaitEvent(streams[0], sum_events[g], 0), "hipStreamWaitEvent");
    }
    const int64_t n4 = (int64_t)count / 4;   // V*Kp + Kp: a multiple of 4 (Kp % 64 == 0)
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((n4 + 255) / 256, 4096));
    for (size_t g = 1; g < G; ++g) {
      hipLaunchKernelGGL(k_sum_into, dim3(blocks), dim3(256), 0, streams[0], static_cast<int4*>(ptr[0]),
                         static_cast<const int4*>(ptr[g]), n4);
      hip_check(hipGetLastError(), "k_sum_into");
    }
    for (size_t g = 1; g < G; ++g)
      hip_check(hipMemcpyAsync(ptr[g], ptr[0], count * sizeof(int32_t), hipMemcpyDeviceToDevice, streams[0]),
                "hipMemcpyAsync");
    hip_check(hipEventRecord(sum_events[0], streams[0]), "hipEventRecord");
    for (size_t g = 1; g < G; ++g) hip_check(hipStreamWaitEvent(streams[g], sum_events[0], 0), "hipStreamWaitEvent");
  }

  hipStream_t stream(size_t g) {
    void* s = nullptr;
    check(lda_get_stream(ctx[g], &s), "lda_get_stream");
    return static_cast<hipStream_t>(s);
  }

  bool use_compact() const { return compact && (!local_sum || local_compact) && ctx.size() > 1; }

  // local_sum + use_compact(): every shard's first n int32 of its escape
  // list copied into every shard's escapes_all [G x n] in shard order (what
  // ncclAllGather leaves on distinct devices)
  void local_gather(int part, size_t n, const std::vector<hipStream_t>& streams) {
    const size_t G = ctx.size();
    for (size_t g = 0; g < G; ++g)
      for (size_t r = 0; r < G; ++r)
        hip_check(hipMemcpyAsync(escapes_all[(size_t)part][g] + r * n, escapes[(size_t)part][r],
                                 sizeof(int32_t) * n, hipMemcpyDeviceToDevice, streams[g]),
                  "hipMemcpyAsync");
  }

  // the compact exchange's cells per packed word and list mode, once the
  // shards exist: four 8-bit cells for the large-K sampler's tables (Kp >=
  // 2048, at most 64 shards) when the lists travel at their used length --
  // C5 at 8 GPUs: 1.07 GB instead of 2.15 GB per exchange, ~1e5 escapes per
  // shard per sweep -- else two (C4: the narrower fields
  // escape about as many bytes as they save).  LDA_ESCAPE_LISTS=capacity
  // and LDA_EXCHANGE_CELLS=2|4 override (A/B and tests).
  void init_cells(int32_t kp) {
    const char* el = std::getenv("LDA_ESCAPE_LISTS");
    used_lists = !(el && std::strcmp(el, "capacity") == 0);
    cells = (used_lists && ctx.size() <= 64 && kp >= 2048) ? 4 : 2;
    const char* ec = std::getenv("LDA_EXCHANGE_CELLS");
    if (ec && (ec[0] == '2' || ec[0] == '4') && ec[1] == 0) cells = ec[0] - '0';
    if (cells == 4 && !used_lists)
      raise(LDA_ERR_UNSUPPORTED, "four cells per word need used-length escape lists (their capacity is "
                                 "three times the two-cell lists')");
    for (auto c : ctx) check(lda_set_exchange_cells(c, cells), "lda_set_exchange_cells");
  }

  // the compact exchange's first step, on every shard's own stream: part
  // `part`'s buffer packed (lda_exchange_pack)
  // escapes_all[part][g] able to hold G x n int32 (grown on demand: with
  // four cells a C5 shard's list capacity is 750 MB, and G copies of it per
  // device would be 6 GB for lists that are normally ~1 MB)
  void reserve_gathered(int part, size_t n) {
    const size_t G = ctx.size();
    if (gathered_cap[(size_t)part] >= n) return;
    const size_t want = std::min(escape_count, std::max(n + n / 2, (size_t)4096));
    for (size_t g = 0; g < G; ++g) {
      hip_check(hipSetDevice(dev[g]), "hipSetDevice");
      if (escapes_all[(size_t)part][g]) {
        // an unpack of an earlier exchange may still read the old lists
        hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize");
        hip_check(hipFree(escapes_all[(size_t)part][g]), "hipFree");
      }
      escapes_all[(size_t)part][g] = nullptr;
      hip_check(hipMalloc(reinterpret_cast<void**>(&escapes_all[(size_t)part][g]), sizeof(int32_t) * want * G),
                "hipMalloc");
    }
    gathered_cap[(size_t)part] = want;
  }

  void pack_part(int part) {
    if (!use_compact()) return;
    const size_t G = ctx.size();
    if (packed.size() <= (size_t)part) {
      packed.resize((size_t)part + 1, std::vector<void*>(G));
      escapes.resize((size_t)part + 1, std::vector<void*>(G));
      escapes_all.resize((size_t)part + 1, std::vector<int32_t*>(G, nullptr));
      gathered_cap.resize((size_t)part + 1, 0);
      part_m.resize((size_t)part + 1, 0);
    }
    check(lda_exchange_sizes(ctx[0], (int32_t)G, max_tokens, &packed_count, &escape_count), "lda_exchange_sizes");
    if (used_lists && !host_counts) {
      hip_check(hipHostMalloc(reinterpret_cast<void**>(&host_counts), sizeof(int32_t) * G * LDA_MAX_EXCHANGE_PARTS,
                              hipHostMallocPortable),
                "hipHostMalloc");
      count_events.assign(LDA_MAX_EXCHANGE_PARTS, std::vector<hipEvent_t>(G, nullptr));
      for (auto& v : count_events)
        for (size_t g = 0; g < G; ++g) {
          hip_check(hipSetDevice(dev[g]), "hipSetDevice");
          hip_check(hipEventCreateWithFlags(&v[g], hipEventDisableTiming), "hipEventCreate");
        }
    }
    for (size_t g = 0; g < G; ++g) {
      check(lda_exchange_pack(ctx[g], part, (int32_t)G, max_tokens, &packed[(size_t)part][g],
                              &escapes[(size_t)part][g]),
            "lda_exchange_pack");
      if (used_lists) {
        // the list's count word to pinned memory behind the pack, on the
        // shard's stream: the host reads it in gather_part
        hip_check(hipSetDevice(dev[g]), "hipSetDevice");
        hip_check(hipMemcpyAsync(host_counts + (size_t)part * G + g, escapes[(size_t)part][g], sizeof(int32_t),
                                 hipMemcpyDeviceToHost, stream(g)),
                  "hipMemcpyAsync");
        hip_check(hipEventRecord(count_events[(size_t)part][g], stream(g)), "hipEventRecord");
      }
    }
    if (!used_lists) reserve_gathered(part, escape_count);
  }

  // the escape lists' all-gather, on streams[g] behind the packed words'
  // sum: the whole lists, or (used_lists) the host reads the counts the pack
  // staged and gathers 1 + 3 m int32 per shard
  void gather_part(int part, const std::vector<hipStream_t>& streams) {
    if (!use_compact()) return;
    const size_t G = ctx.size();
    size_t n = escape_count;
    if (used_lists) {
      int32_t m = 0;
      for (size_t g = 0; g < G; ++g) {
        hip_check(hipEventSynchronize(count_events[(size_t)part][g]), "hipEventSynchronize");
        m = std::max(m, host_counts[(size_t)part * G + g]);
      }
      const int32_t cap = (int32_t)((escape_count - 1) / 3);
      if (m < 0 || m > cap)
        raise(LDA_ERR_STATE, "escape list overflow: " + std::to_string(m) + " escapes, capacity " +
                                 std::to_string(cap));
      part_m[(size_t)part] = m;
      m_max = std::max(m_max, m);
      ++list_exchanges;
      if (m == 0) return;
      n = 1 + 3 * (size_t)m;
      reserve_gathered(part, n);
    }
    if (local_sum) {
      local_gather(part, n, streams);
      return;
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t g = 0; g < G && r == ncclSuccess; ++g)
      r = ncclAllGather(escapes[(size_t)part][g], escapes_all[(size_t)part][g], n, ncclInt32, comms[g], streams[g]);
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      raise(LDA_ERR_DEVICE, std::string("ncclAllGather: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  }

  // ... and its last, on every shard's own stream: the part's buffer = the sum
  void unpack_part(int part) {
    if (!use_compact()) return;
    const int32_t G = (int32_t)ctx.size();
    for (size_t g = 0; g < ctx.size(); ++g) {
      if (used_lists) {
        const int32_t m = part_m[(size_t)part];
        check(lda_exchange_unpack_lists(ctx[g], part, G, max_tokens, m ? escapes_all[(size_t)part][g] : nullptr, m),
              "lda_exchange_unpack_lists");
      } else {
        check(lda_exchange_unpack(ctx[g], part, G, max_tokens, escapes_all[(size_t)part][g]),
              "lda_exchange_unpack");
      }
    }
  }

  // the sum of part `part`'s buffers across the shards, each shard's on
  // streams[g] (its own stream, or its collective stream): compact, one
  // grouped SUM all-reduce of the packed words (pack_part before,
  // gather_part and unpack_part after); or the int32 buffers themselves
  // (all-reduce / the device-side sum)
  void reduce_part(int part, const std::vector<hipStream_t>& streams) {
    std::vector<void*> ptr(ctx.size());
    size_t count = 0;
    for (size_t g = 0; g < ctx.size(); ++g)
      check(lda_delta_buffer_part(ctx[g], part, &ptr[g], &count), "lda_delta_buffer_part");
    const bool cmp = use_compact();
    if (local_sum) {
      if (cmp)
        local_reduce(packed[(size_t)part], packed_count, streams);   // a multiple of 4 int32
      else
        local_reduce(ptr, count, streams);
      return;
    }
    ncclResult_t r = ncclGroupStart();
    for (size_t g = 0; g < ctx.size() && r == ncclSuccess; ++g) {
      if (cmp) {
        void* pk = packed[(size_t)part][g];
        r = ncclAllReduce(pk, pk, packed_count, ncclInt32, ncclSum, comms[g], streams[g]);
      } else {
        r = ncclAllReduce(ptr[g], ptr[g], count, ncclInt32, ncclSum, comms[g], streams[g]);
      }
    }
    const ncclResult_t r2 = ncclGroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess)
      raise(LDA_ERR_DEVICE, std::string("ncclAllReduce: ") + ncclGetErrorString(r != ncclSuccess ? r : r2));
  }

  void reduce() {
    if (ctx.size() < 2) return;
    std::vector<hipStream_t> st(ctx.size());
    for (size_t g = 0; g < ctx.size(); ++g) st[g] = stream(g);
    pack_part(0);
    reduce_part(0, st);
    gather_part(0, st);
    unpack_part(0);
  }

  void set_parts(int p) {
    parts = ctx.size() < 2 ? 1 : p;   // nothing to overlap on one GPU
    // reserve_cus < 0: the library's default share of CUs left to the collective
    for (auto c : ctx) check(lda_set_exchange_parts(c, parts, parts > 1 ? -1 : 0), "lda_set_exchange_parts");
    if (parts > 1 && comm_streams.empty()) {
      comm_streams.resize(ctx.size());
      events.resize(ctx.size());
      for (size_t g = 0; g < ctx.size(); ++g) {
        if (hipSetDevice(dev[g]) != hipSuccess ||
            hipStreamCreateWithFlags(&comm_streams[g], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&events[g], hipEventDisableTiming) != hipSuccess)
          raise(LDA_ERR_DEVICE, "collective stream");
      }
    }
  }

  // sample + exchange + apply of one sweep
  void sweep() {
    int32_t np = 1, seq = 0;
    check(lda_sweep_parts(ctx[0], &np, &seq), "lda_sweep_parts");
    if (seq) {
      // a warm-start sweep: every part sampled, summed and applied in turn
      for (int i = 0; i < np; ++i) {
        for (auto c : ctx) check(lda_sample_part(c, i), "lda_sample_part");
        reduce();
        apply();
      }
      return;
    }
    if (ctx.size() < 2 || parts < 2) {
      for (auto c : ctx) check(lda_sample(c), "lda_sample");
      reduce();
      apply();
      return;
    }
    std::vector<hipStream_t> st(ctx.size());
    for (size_t g = 0; g < ctx.size(); ++g) st[g] = stream(g);
    auto hip = [](hipError_t e, const char* what) {
      if (e != hipSuccess) raise(LDA_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
    };
    for (int i = 0; i < parts; ++i) {
      for (size_t g = 0; g < ctx.size(); ++g) check(lda_sample_part(ctx[g], i), "lda_sample_part");
      pack_part(i);                       // on the shards' streams, before the event
      for (size_t g = 0; g < ctx.size(); ++g) {
        hip(hipSetDevice(dev[g]), "hipSetDevice");
        hip(hipEventRecord(events[g], st[g]), "hipEventRecord");           // part i sampled
        hip(hipStreamWaitEvent(comm_streams[g], events[g], 0), "hipStreamWaitEvent");
      }
      reduce_part(i, comm_streams);
    }
    // every part's escape lists once every sampler part is enqueued: the
    // count reads wait for the parts' packs, not for the packed sums
    for (int i = 0; i < parts; ++i) gather_part(i, comm_streams);
    for (size_t g = 0; g < ctx.size(); ++g) {
      hip(hipSetDevice(dev[g]), "hipSetDevice");
      hip(hipEventRecord(events[g], comm_streams[g]), "hipEventRecord");   // every sum landed
      hip(hipStreamWaitEvent(st[g], events[g], 0), "hipStreamWaitEvent");
    }
    for (int i = 0; i < parts; ++i) unpack_part(i);
    apply();
  }
  void apply() {
    for (auto c : ctx) check(lda_apply(c), "lda_apply");
  }
  // n sweeps; one shard runs them through lda_sweep, which launches plain
  // sweeps as graphs (the reference's small corpora are launch-bound)
  void sweeps(int32_t n) {
    if (ctx.size() == 1) {
      check(lda_sweep(ctx[0], n), "lda_sweep");
      return;
    }
    for (int32_t i = 0; i < n; ++i) sweep();
  }
};

// ------------------------------------------------------------------ model
ParallelTopicModel::ParallelTopicModel(int32_t num_topics, double alpha_sum, double beta)
    : K_(num_topics), alpha_sum_(alpha_sum), beta_(beta) {
  if (num_topics < 1 || num_topics > LDA_MAX_TOPICS) raise(LDA_ERR_UNSUPPORTED, "num_topics out of range");
  if (!(alpha_sum > 0.0) || !(beta > 0.0)) raise(LDA_ERR_INVALID_ARG, "alphaSum and beta must be > 0");
  alpha_.assign((size_t)K_, alpha_sum / K_);
  // the dense sampler holds K <= 1024; above that the large-K sparse one
  sampler_ = K_ > LDA_MAX_TOPICS_DENSE ? LDA_SAMPLER_SPARSE : LDA_SAMPLER_DENSE;
}

void ParallelTopicModel::setTopics(const int32_t* z, int64_t n) {
  if (n != numTokens()) raise(LDA_ERR_INVALID_ARG, "setTopics needs one topic per token");
  for (int64_t i = 0; i < n; ++i)
    if (z[i] < 0 || z[i] >= K_) raise(LDA_ERR_INVALID_ARG, "topic out of range [0, K)");
  markDirty();
  z_cache_.assign(z, z + n);
}

void ParallelTopicModel::setHyper(const double* alpha, double alpha_sum, double beta) {
  for (int k = 0; k < K_; ++k)
    if (!(alpha[k] > 0.0)) raise(LDA_ERR_INVALID_ARG, "alpha must be > 0");
  if (!(beta > 0.0) || !(alpha_sum > 0.0)) raise(LDA_ERR_INVALID_ARG, "alphaSum and beta must be > 0");
  alpha_.assign(alpha, alpha + K_);
  alpha_sum_ = alpha_sum;
  beta_ = beta;
  if (shards_ && !shards_dirty_)
    for (auto c : shards_->ctx) check(lda_set_alpha_beta(c, alpha_.data(), beta_), "lda_set_alpha_beta");
}

uint32_t ParallelTopicModel::sweep() {
  if (shards_ && !shards_dirty_) check(lda_get_sweep(shards_->ctx[0], &sweep_), "lda_get_sweep");
  return sweep_;
}

void ParallelTopicModel::setSweep(uint32_t s) {
  sweep_ = s;
  if (shards_ && !shards_dirty_)
    for (auto c : shards_->ctx) check(lda_set_sweep(c, sweep_), "lda_set_sweep");
}

ParallelTopicModel::~ParallelTopicModel() = default;

// Anything that invalidates the GPU shards first saves the current topic
// assignments (documents keep their z across re-sharding / addInstances).
void ParallelTopicModel::markDirty() {
  if (shards_ && !shards_dirty_) {
    z_cache_ = topics();
    check(lda_get_sweep(shards_->ctx[0], &sweep_), "lda_get_sweep");
  }
  shards_dirty_ = true;
}

void ParallelTopicModel::setRandomSeed(int64_t seed) {
  markDirty();
  seed_ = (uint64_t)seed;
}

void ParallelTopicModel::setNumThreads(int32_t n) {
  if (n < 1) raise(LDA_ERR_INVALID_ARG, "numThreads must be >= 1");
  markDirty();
  num_threads_ = n;
}

void ParallelTopicModel::setWarmStart(int32_t parts, int32_t sweeps) {
  if (parts < 1 || parts > LDA_MAX_EXCHANGE_PARTS || sweeps < 0)
    raise(LDA_ERR_INVALID_ARG, "warm start: parts in [1, 4], sweeps >= 0");
  warm_parts_ = parts;
  warm_sweeps_ = sweeps;
  if (shards_ && !shards_dirty_) applySweepSchedule();
}

void ParallelTopicModel::setStalenessThreads(int32_t threads) {
  staleness_threads_ = threads;
  if (shards_ && !shards_dirty_) applySweepSchedule();
}

// the shards' sequential sweeps: the warm start, then Mallet's staleness for
// T threads; parts cut in the whole corpus, so the sweeps are
// the same for any shard count
void ParallelTopicModel::applySweepSchedule() {
  const int64_t N = numTokens();
  int32_t parts = 1;
  double fr[LDA_MAX_EXCHANGE_PARTS] = {1.0};
  const int32_t T = staleness_threads_ == 0 ? num_threads_ : staleness_threads_;
  if (T > 0) check(lda_staleness_schedule(T, &parts, fr), "lda_staleness_schedule");
  for (auto c : shards_->ctx) {
    check(lda_set_warm_start(c, warm_parts_, warm_sweeps_, 0, N), "lda_set_warm_start");
    check(lda_set_sequential_sweeps(c, parts, parts > 1 ? fr : nullptr, 0, N), "lda_set_sequential_sweeps");
  }
}

void ParallelTopicModel::setDevices(const int32_t* devices, int32_t n) {
  if (n < 0 || (n > 0 && !devices)) raise(LDA_ERR_INVALID_ARG, "setDevices: bad argument");
  devices_.assign(devices, devices + n);
  markDirty();
}

int32_t ParallelTopicModel::numShards() {
  ensureShards();
  return (int32_t)shards_->ctx.size();
}

void ParallelTopicModel::exchangeInfo(int32_t* cells, int32_t* used_lists, int32_t* escapes_max,
                                      int64_t* list_exchanges) {
  ensureShards();
  const ShardGroup& s = *shards_;
  const bool cmp = s.use_compact();
  if (cells) *cells = cmp ? s.cells : 0;
  if (used_lists) *used_lists = cmp && s.used_lists ? 1 : 0;
  if (escapes_max) *escapes_max = s.m_max;
  if (list_exchanges) *list_exchanges = s.list_exchanges;
}

void ParallelTopicModel::setExchangeParts(int32_t parts) {
  if (parts < 1 || parts > LDA_MAX_EXCHANGE_PARTS) raise(LDA_ERR_INVALID_ARG, "parts out of range");
  exchange_parts_ = parts;
  if (shards_ && !shards_dirty_) shards_->set_parts(parts);
}

void ParallelTopicModel::setSampler(int32_t sampler) {
  if (sampler != LDA_SAMPLER_DENSE && sampler != LDA_SAMPLER_SPARSE)
    raise(LDA_ERR_INVALID_ARG, "unknown sampler");
  markDirty();
  sampler_ = sampler;
}

void ParallelTopicModel::setAlphabet(std::vector<std::string> words, int32_t num_types) {
  if (num_types < V_) raise(LDA_ERR_INVALID_ARG, "the alphabet cannot shrink");
  if (!words.empty() && (int32_t)words.size() != num_types)
    raise(LDA_ERR_INVALID_ARG, "alphabet size mismatch");
  if (num_types != V_) markDirty();
  alphabet_ = std::move(words);
  V_ = num_types;
}

void ParallelTopicModel::addInstances(int64_t D, const int64_t* doc_off, const int32_t* words,
                                      const char* const* sources) {
  if (D < 0 || (D > 0 && !doc_off)) raise(LDA_ERR_INVALID_ARG, "bad documents");
  if (V_ < 1) raise(LDA_ERR_STATE, "set the alphabet before addInstances");
  markDirty();  // documents already in the model keep their z
  const int64_t base = doc_off_.back();
  for (int64_t d = 0; d < D; ++d) {
    const int64_t a = doc_off[d] - doc_off[0], b = doc_off[d + 1] - doc_off[0];
    if (b < a) raise(LDA_ERR_INVALID_ARG, "doc_off not monotone");
    for (int64_t i = a; i < b; ++i) {
      if (words[i] < 0 || words[i] >= V_) raise(LDA_ERR_INVALID_ARG, "word id outside the alphabet");
      words_.push_back(words[i]);
    }
    doc_off_.push_back(base + b);
    const bool has = sources && sources[d];
    sources_.push_back(has ? sources[d] : "");
    has_source_.push_back(has ? 1 : 0);
  }
}

void ParallelTopicModel::log(const std::string& line) const {
  if (verbosity_ > 0) {
    std::fputs(line.c_str(), stderr);
    std::fputc('\n', stderr);
  }
}

void ParallelTopicModel::ensureShards() {
  if (shards_ && !shards_dirty_) return;
  if (V_ < 1) raise(LDA_ERR_STATE, "no alphabet: call addInstances first");
  const std::vector<int32_t> keep = z_cache_;  // saved by markDirty (may be shorter than N)
  shards_.reset();
  const int64_t D = numDocs(), N = numTokens();
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) raise(LDA_ERR_DEVICE, "no HIP device");
  // explicit placement (setDevices) or setNumThreads' plan
  const int G = devices_.empty() ? plan_shards(num_threads_, ndev, N, V_, K_, D)
                                 : (int)std::min<int64_t>((int64_t)devices_.size(), std::max<int64_t>(D, 1));
  for (int32_t d : devices_)
    if (d < 0 || d >= ndev) raise(LDA_ERR_INVALID_ARG, "setDevices: device ordinal out of range");
  auto sg = std::make_unique<ShardGroup>();
  for (int g = 0; g < G; ++g) sg->dev.push_back(devices_.empty() ? g : devices_[(size_t)g]);
  // token-balanced contiguous document ranges (the cuts Mallet makes by
  // document count; tokens balance the GPUs' work)
  sg->doc_begin.push_back(0);
  for (int g = 1; g < G; ++g) {
    const int64_t target = N * g / G;
    int64_t d = std::lower_bound(doc_off_.begin(), doc_off_.end(), target) - doc_off_.begin();
    d = std::max(d, sg->doc_begin.back());
    sg->doc_begin.push_back(std::min(d, D));
  }
  sg->doc_begin.push_back(D);
  for (int g = 0; g < G; ++g) {
    const int64_t d0 = sg->doc_begin[g], d1 = sg->doc_begin[g + 1];
    lda_config cfg{};
    cfg.num_topics = K_;
    cfg.num_types = V_;
    cfg.num_docs = d1 - d0;
    cfg.alpha = alpha_.data();
    cfg.beta = beta_;
    cfg.seed = seed_;
    cfg.device = sg->dev[(size_t)g];
    cfg.sampler = sampler_;
    cfg.token_base = doc_off_[d0];
    cfg.tokens_per_range = 0;
    lda_ctx* c = nullptr;
    const int32_t* w = words_.empty() ? nullptr : words_.data() + doc_off_[d0];
    check(lda_create(&c, &cfg, doc_off_.data() + d0, w, nullptr), "lda_create");
    sg->ctx.push_back(c);
  }
  // documents already in the model keep their topics
  if (!keep.empty()) {
    for (int g = 0; g < G; ++g) {
      const int64_t t0 = doc_off_[sg->doc_begin[g]], t1 = doc_off_[sg->doc_begin[g + 1]];
      if (t0 >= (int64_t)keep.size() || t1 == t0) continue;
      std::vector<int32_t> z((size_t)(t1 - t0));
      check(lda_get_z(sg->ctx[g], z.data()), "lda_get_z");
      const int64_t m = std::min<int64_t>(t1, (int64_t)keep.size());
      std::copy(keep.begin() + t0, keep.begin() + m, z.begin());
      check(lda_set_z(sg->ctx[g], z.data()), "lda_set_z");
    }
  }
  sg->init_exchange();
  for (int g = 0; g < G; ++g)
    sg->max_tokens = std::max(sg->max_tokens, doc_off_[sg->doc_begin[(size_t)g + 1]] - doc_off_[sg->doc_begin[(size_t)g]]);
  {
    const char* e = std::getenv("LDA_EXCHANGE_INT32");
    sg->compact = compact_exchange_ && !(e && e[0] == '1');
    const char* lc = std::getenv("LDA_LOCAL_COMPACT");
    sg->local_compact = lc && lc[0] == '1';
    if (sg->use_compact()) sg->init_cells(lda_padded_topics(K_));
  }
  if (G > 1) {
    // shards recount (or keep a delta) in the same sweeps: the smallest
    // AUTO recount count of any shard on all of them
    int32_t rmin = INT32_MAX;
    for (auto c : sg->ctx) {
      int32_t mode = 0, r = 0;
      check(lda_get_count_update(c, &mode, &r), "lda_get_count_update");
      rmin = std::min(rmin, r);
    }
    for (auto c : sg->ctx) {
      int32_t mode = 0;
      check(lda_get_count_update(c, &mode, nullptr), "lda_get_count_update");
      if (mode == LDA_COUNT_AUTO) check(lda_set_count_update(c, LDA_COUNT_AUTO, rmin), "lda_set_count_update");
    }
  }
  // the shards' local counts are the pending delta: sum them, apply
  sg->reduce();
  sg->apply();
  sg->set_parts(exchange_parts_);
  for (auto c : sg->ctx) check(lda_set_sweep(c, sweep_), "lda_set_sweep");
  shards_ = std::move(sg);
  applySweepSchedule();
  shards_dirty_ = false;
  z_dirty_ = true;
  // word totals never change between addInstances calls: the bound of beta's
  // countHistogram is taken once here, not by an O(N) pass per optimisation
  {
    std::vector<int32_t> totals((size_t)V_, 0);
    for (int32_t w : words_) totals[(size_t)w]++;
    max_word_total_ = totals.empty() ? 0 : *std::max_element(totals.begin(), totals.end());
  }
  int32_t m = 0;
  for (int64_t d = 0; d < D; ++d) m = std::max<int32_t>(m, (int32_t)(doc_off_[d + 1] - doc_off_[d]));
  if (m != max_doc_len_) {  // statistics gathered so far stay valid unless the shape changes
    max_doc_len_ = m;
    doc_len_counts_.assign((size_t)max_doc_len_ + 1, 0);
    topic_doc_counts_.assign((size_t)K_ * (max_doc_len_ + 1), 0);
  }
}

std::vector<int32_t> ParallelTopicModel::topics() {
  ensureShards();  // documents added since the last sweep get their initial topics
  if (z_dirty_) {
    z_cache_.assign((size_t)numTokens(), 0);
    for (size_t g = 0; g < shards_->ctx.size(); ++g) {
      const int64_t t0 = doc_off_[shards_->doc_begin[g]];
      check(lda_get_z(shards_->ctx[g], z_cache_.data() + t0), "lda_get_z");
    }
    z_dirty_ = false;
  }
  return z_cache_;
}

void ParallelTopicModel::counts(int32_t* nw, int32_t* nwsum) {
  ensureShards();
  check(lda_get_counts(shards_->ctx[0], nw, nwsum, nullptr, nullptr), "lda_get_counts");
}

double ParallelTopicModel::modelLogLikelihood() {
  ensureShards();
  double doc_total = 0.0, word_part = 0.0;
  for (size_t g = 0; g < shards_->ctx.size(); ++g) {
    double dp = 0.0, wp = 0.0;
    check(lda_log_likelihood_parts(shards_->ctx[g], &dp, &wp), "lda_log_likelihood_parts");
    doc_total += dp;
    if (g == 0) word_part = wp;
  }
  return doc_total + word_part;
}

void ParallelTopicModel::optimizeAlpha() {
  const int64_t W = (int64_t)max_doc_len_ + 1;
  if (symmetric_alpha_) {
    // every topic's histogram pooled into one (Mallet keeps it in topic 0's row)
    std::vector<int32_t> pooled((size_t)W, 0);
    for (int k = 0; k < K_; ++k)
      for (int64_t i = 0; i < W; ++i) pooled[(size_t)i] += topic_doc_counts_[(size_t)(k * W + i)];
    std::vector<int64_t> lens;
    std::vector<int32_t> cnt;
    for (int64_t n = 0; n < W; ++n)
      if (doc_len_counts_[(size_t)n] > 0) {
        lens.push_back(n);
        cnt.push_back(doc_len_counts_[(size_t)n]);
      }
    double a = 0.0;
    check(lda_learn_symmetric_concentration(pooled.data(), W - 1, lens.data(), cnt.data(),
                                            (int64_t)lens.size(), K_, alpha_sum_, &a),
          "lda_learn_symmetric_concentration");
    alpha_sum_ = a;
    std::fill(alpha_.begin(), alpha_.end(), alpha_sum_ / K_);
  } else {
    double s = 0.0;
    check(lda_learn_parameters(alpha_.data(), K_, topic_doc_counts_.data(), doc_len_counts_.data(),
                               max_doc_len_, 1.001, 1.0, 1, &s),
          "lda_learn_parameters");
    alpha_sum_ = s;
  }
  std::fill(doc_len_counts_.begin(), doc_len_counts_.end(), 0);
  std::fill(topic_doc_counts_.begin(), topic_doc_counts_.end(), 0);
}

void ParallelTopicModel::optimizeBeta(const std::vector<int32_t>& hist, const std::vector<int32_t>& nwsum) {
  // countHistogram: nw cells by count, up to the largest word total (hist);
  // topicSizeHistogram, sparse: (tokens in topic, number of topics)
  const int64_t max_count = max_word_total_;
  std::vector<int64_t> sizes(nwsum.begin(), nwsum.end());
  std::sort(sizes.begin(), sizes.end());
  std::vector<int64_t> lens;
  std::vector<int32_t> cnt;
  for (int64_t s : sizes) {
    if (!lens.empty() && lens.back() == s) {
      cnt.back()++;
    } else {
      lens.push_back(s);
      cnt.push_back(1);
    }
  }
  double beta_sum = beta_ * V_;
  check(lda_learn_symmetric_concentration(hist.data(), max_count, lens.data(), cnt.data(),
                                          (int64_t)lens.size(), V_, beta_sum, &beta_sum),
        "lda_learn_symmetric_concentration");
  beta_ = beta_sum / V_;
}

void ParallelTopicModel::estimate() {
  ensureShards();
  ll_trace_.clear();
  const double total_tokens = (double)numTokens();
  // Mallet's estimate() builds new WorkerRunnables whose alpha statistics
  // start empty (WorkerRunnable.initializeAlphaStatistics): statistics still
  // pending from an earlier estimate() are not carried into this one
  std::fill(doc_len_counts_.begin(), doc_len_counts_.end(), 0);
  std::fill(topic_doc_counts_.begin(), topic_doc_counts_.end(), 0);
  for (auto c : shards_->ctx) check(lda_doc_topic_histograms_clear(c), "lda_doc_topic_histograms_clear");
  // LL/token every 10 sweeps without stopping the sweeps: the kernels are
  // enqueued behind the sweep and their sums collected (and logged) in
  // batches, and at the end
  std::vector<std::pair<int32_t, std::vector<int64_t>>> ll_pending;
  auto collect_ll = [&]() {
    for (const auto& p : ll_pending) {
      double ll = 0.0;
      for (size_t g = 0; g < shards_->ctx.size(); ++g) {
        double dp = 0.0, wp = 0.0;
        check(lda_log_likelihood_collect(shards_->ctx[g], p.second[g], &dp, &wp), "lda_log_likelihood_collect");
        ll += dp + (g == 0 ? wp : 0.0);   // the word part is global: once
      }
      ll /= total_tokens;
      ll_trace_.emplace_back(p.first, ll);
      log("<" + std::to_string(p.first) + "> LL/token: " + java_number5(ll));
    }
    ll_pending.clear();
  };
  // iterations after which something besides the sweep happens (statistics,
  // optimisation, LL), or before which the topics are shown: the sweeps in
  // between run as one batch
  auto work_after = [&](int32_t i) {
    const bool opt = i > burnin_period_ && optimize_interval_ != 0;
    return i % 10 == 0 || (opt && (i % save_sample_interval_ == 0 || i % optimize_interval_ == 0));
  };
  auto show_before = [&](int32_t i) { return show_topics_interval_ != 0 && i % show_topics_interval_ == 0; };
  for (int32_t it = 1; it <= num_iterations_; ++it) {
    if (show_before(it)) {
      collect_ll();
      log("\n" + displayTopWords(words_per_topic_, false));
    }
    int32_t last = it;
    while (last < num_iterations_ && !work_after(last) && !show_before(last + 1)) ++last;
    shards_->sweeps(last - it + 1);
    it = last;
    z_dirty_ = true;
    const bool opt = it > burnin_period_ && optimize_interval_ != 0;
    if (opt && it % save_sample_interval_ == 0)
      for (auto c : shards_->ctx)
        check(lda_doc_topic_histograms_accumulate(c, max_doc_len_), "lda_doc_topic_histograms_accumulate");
    if (opt && it % optimize_interval_ == 0) {
      // every shard's alpha statistics (summed); the count histogram and
      // nwsum of the global counts from shard 0; one wait per shard
      std::vector<int32_t> hist((size_t)max_word_total_ + 1, 0), nwsum((size_t)K_);
      for (size_t g = 0; g < shards_->ctx.size(); ++g)
        check(lda_hyper_statistics(shards_->ctx[g], max_doc_len_, doc_len_counts_.data(), topic_doc_counts_.data(),
                                   max_word_total_, g == 0 ? hist.data() : nullptr,
                                   g == 0 ? nwsum.data() : nullptr),
              "lda_hyper_statistics");
      optimizeAlpha();
      optimizeBeta(hist, nwsum);
      for (auto c : shards_->ctx) check(lda_set_alpha_beta(c, alpha_.data(), beta_), "lda_set_alpha_beta");
    }
    if (it % 10 == 0) {
      if (print_log_likelihood_) {
        std::vector<int64_t> tickets(shards_->ctx.size());
        for (size_t g = 0; g < shards_->ctx.size(); ++g)
          check(lda_log_likelihood_enqueue(shards_->ctx[g], &tickets[g]), "lda_log_likelihood_enqueue");
        ll_pending.emplace_back(it, std::move(tickets));
        if (ll_pending.size() >= 8) collect_ll();
      } else {
        log("<" + std::to_string(it) + ">");
      }
    }
  }
  collect_ll();
  // statistics gathered after the last optimisation are dropped, as Mallet's
  // runnables are
  for (auto c : shards_->ctx) check(lda_doc_topic_histograms_clear(c), "lda_doc_topic_histograms_clear");
  // Mallet's estimate() returns when the sweeps are done: wait for the shards'
  // streams (a kernel fault surfaces here, not in a later call)
  for (auto c : shards_->ctx) check(lda_synchronize(c), "lda_synchronize");
}

std::vector<double> ParallelTopicModel::getTopicProbabilities(int64_t doc) {
  if (doc < 0 || doc >= numDocs()) raise(LDA_ERR_INVALID_ARG, "document index out of range");
  ensureShards();
  const std::vector<int32_t> z = topics();
  std::vector<double> dist((size_t)K_, 0.0);
  for (int64_t i = doc_off_[doc]; i < doc_off_[doc + 1]; ++i) dist[(size_t)z[(size_t)i]] += 1.0;
  double sum = 0.0;
  for (int k = 0; k < K_; ++k) {
    dist[(size_t)k] += alpha_[(size_t)k];
    sum += dist[(size_t)k];
  }
  for (int k = 0; k < K_; ++k) dist[(size_t)k] /= sum;
  return dist;
}

// IDSorter order: weight descending; equal weights by ascending id (Mallet's
// stable sort of an array already in id order; parity unpinned)
static void sort_ids(std::vector<std::pair<int32_t, double>>& v) {
  std::stable_sort(v.begin(), v.end(), [](const auto& a, const auto& b) { return a.second > b.second; });
}

std::string ParallelTopicModel::documentTopics(double threshold, int32_t max) {
  ensureShards();
  const std::vector<int32_t> z = topics();
  if (max < 0 || max > K_) max = K_;
  std::string out = "#doc source topic proportion ...\n";
  std::vector<int32_t> cnt((size_t)K_);
  std::vector<std::pair<int32_t, double>> sorted((size_t)K_);
  for (int64_t d = 0; d < numDocs(); ++d) {
    out += std::to_string(d);
    out += ' ';
    out += has_source_[(size_t)d] ? sources_[(size_t)d] : std::string("null-source");
    out += ' ';
    std::fill(cnt.begin(), cnt.end(), 0);
    const int64_t len = doc_off_[d + 1] - doc_off_[d];
    for (int64_t i = doc_off_[d]; i < doc_off_[d + 1]; ++i) cnt[(size_t)z[(size_t)i]]++;
    for (int k = 0; k < K_; ++k)
      sorted[(size_t)k] = {k, (alpha_[(size_t)k] + cnt[(size_t)k]) / ((double)len + alpha_sum_)};
    sort_ids(sorted);
    for (int i = 0; i < max; ++i) {
      if (sorted[(size_t)i].second < threshold) break;
      out += std::to_string(sorted[(size_t)i].first) + " " + java_double(sorted[(size_t)i].second) + " ";
    }
    out += " \n";
  }
  return out;
}

std::string ParallelTopicModel::displayTopWords(int32_t num_words, bool using_new_lines) {
  ensureShards();
  std::vector<int32_t> nw((size_t)V_ * K_);
  check(lda_get_counts(shards_->ctx[0], nw.data(), nullptr, nullptr, nullptr), "lda_get_counts");
  std::string out;
  std::vector<std::pair<int32_t, double>> words;
  for (int k = 0; k < K_; ++k) {
    words.clear();
    for (int32_t w = 0; w < V_; ++w) {
      const int32_t c = nw[(size_t)w * K_ + k];
      if (c > 0) words.emplace_back(w, (double)c);
    }
    sort_ids(words);
    auto name = [&](int32_t w) { return alphabet_.empty() ? std::to_string(w) : alphabet_[(size_t)w]; };
    // Mallet's loop starts its word counter at 1 and stops before numWords
    const size_t n = (size_t)std::max(0, std::min<int32_t>(num_words - 1, (int32_t)words.size()));
    if (using_new_lines) {
      out += std::to_string(k) + "\t" + java_number5(alpha_[(size_t)k]) + "\n";
      for (size_t i = 0; i < n; ++i)
        out += name(words[i].first) + "\t" + java_number5(words[i].second) + "\n";
    } else {
      out += std::to_string(k) + "\t" + java_number5(alpha_[(size_t)k]) + "\t";
      for (size_t i = 0; i < n; ++i) out += name(words[i].first) + " ";
      out += "\n";
    }
  }
  return out;
}

// ---- checkpoint: little-endian binary, every field needed to continue the
// run bit for bit (topics, hyperparameters, options and the Philox sweep
// counter).  The alpha statistics arrays are still written (format v2) but
// carry nothing across: estimate() clears them at its start and end, as
// Mallet 2.0.7's new WorkerRunnables drop theirs, so a resumed model starts
// its statistics empty whatever the file holds.
namespace {
// v4: without the alpha-statistics histograms (estimate() starts them
// empty, as Mallet's new WorkerRunnables do, so a file never needs them)
constexpr char kMagic[8] = {'L', 'D', 'A', 'T', 'M', 0, 'v', '4'};
constexpr char kMagicV3[8] = {'L', 'D', 'A', 'T', 'M', 0, 'v', '3'};  // v3: + staleness threads
constexpr char kMagicV2[8] = {'L', 'D', 'A', 'T', 'M', 0, 'v', '2'};  // v2: + warm start
constexpr char kMagicV1[8] = {'L', 'D', 'A', 'T', 'M', 0, 'v', '1'};

struct Writer {
  std::ofstream f;
  template <typename T>
  void pod(const T& v) { f.write(reinterpret_cast<const char*>(&v), sizeof(T)); }
  template <typename T>
  void vec(const std::vector<T>& v) {
    pod<int64_t>((int64_t)v.size());
    if (!v.empty()) f.write(reinterpret_cast<const char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
  }
  void str(const std::string& s) {
    pod<int64_t>((int64_t)s.size());
    f.write(s.data(), (std::streamsize)s.size());
  }
};

struct Reader {
  std::ifstream f;
  template <typename T>
  T pod() {
    T v{};
    f.read(reinterpret_cast<char*>(&v), sizeof(T));
    if (!f) raise(LDA_ERR_INVALID_ARG, "checkpoint truncated");
    return v;
  }
  int64_t count(int64_t limit) {
    const int64_t n = pod<int64_t>();
    if (n < 0 || n > limit) raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (bad length)");
    return n;
  }
  template <typename T>
  std::vector<T> vec(int64_t limit) {
    std::vector<T> v((size_t)count(limit));
    if (!v.empty()) f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(v.size() * sizeof(T)));
    if (!f) raise(LDA_ERR_INVALID_ARG, "checkpoint truncated");
    return v;
  }
  std::string str() {
    std::string s((size_t)count(1 << 30), '\0');
    f.read(&s[0], (std::streamsize)s.size());
    if (!f) raise(LDA_ERR_INVALID_ARG, "checkpoint truncated");
    return s;
  }
};
}  // namespace

void ParallelTopicModel::save(const std::string& path) {
  // live shards: their state; otherwise the snapshot (possibly no topics yet:
  // a model saved before its first use re-initialises them on load)
  const bool live = shards_ && !shards_dirty_;
  const std::vector<int32_t> z = live ? topics() : z_cache_;
  if (live) check(lda_get_sweep(shards_->ctx[0], &sweep_), "lda_get_sweep");
  Writer w{std::ofstream(path, std::ios::binary)};
  if (!w.f) raise(LDA_ERR_INVALID_ARG, "cannot open " + path);
  w.f.write(kMagic, 8);
  w.pod(K_);
  w.pod(V_);
  w.pod(alpha_sum_);
  w.pod(beta_);
  w.vec(alpha_);
  w.pod(seed_);
  w.pod(sweep_);
  for (int32_t v : {num_iterations_, optimize_interval_, burnin_period_, save_sample_interval_,
                    show_topics_interval_, words_per_topic_, (int32_t)symmetric_alpha_,
                    (int32_t)print_log_likelihood_, num_threads_, sampler_})
    w.pod(v);
  w.vec(doc_off_);
  w.vec(words_);
  w.vec(z);
  w.pod<int64_t>((int64_t)alphabet_.size());
  for (const auto& a : alphabet_) w.str(a);
  w.vec(has_source_);
  for (const auto& src : sources_) w.str(src);
  w.pod(max_doc_len_);
  w.pod(warm_parts_);
  w.pod(warm_sweeps_);
  w.pod(staleness_threads_);
  w.f.flush();
  if (!w.f) raise(LDA_ERR_INVALID_ARG, "write failed: " + path);
}

std::unique_ptr<ParallelTopicModel> ParallelTopicModel::load(const std::string& path) {
  Reader r{std::ifstream(path, std::ios::binary)};
  if (!r.f) raise(LDA_ERR_INVALID_ARG, "cannot open " + path);
  char magic[8];
  r.f.read(magic, 8);
  const bool v1 = r.f && std::memcmp(magic, kMagicV1, 8) == 0;
  const bool v2 = r.f && std::memcmp(magic, kMagicV2, 8) == 0;
  const bool v3 = r.f && std::memcmp(magic, kMagicV3, 8) == 0;
  if (!r.f || (!v1 && !v2 && !v3 && std::memcmp(magic, kMagic, 8) != 0))
    raise(LDA_ERR_INVALID_ARG, "not an lda_topic_model checkpoint");
  const int32_t K = r.pod<int32_t>(), V = r.pod<int32_t>();
  const double alpha_sum = r.pod<double>(), beta = r.pod<double>();
  auto m = std::make_unique<ParallelTopicModel>(K, alpha_sum, beta);
  m->V_ = V;
  m->alpha_ = r.vec<double>(K);
  if ((int32_t)m->alpha_.size() != K) raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (alpha)");
  m->seed_ = r.pod<uint64_t>();
  m->sweep_ = r.pod<uint32_t>();
  int32_t opt[10];
  for (int32_t& v : opt) v = r.pod<int32_t>();
  m->num_iterations_ = opt[0];
  m->optimize_interval_ = opt[1];
  m->burnin_period_ = opt[2];
  m->save_sample_interval_ = opt[3];
  m->show_topics_interval_ = opt[4];
  m->words_per_topic_ = opt[5];
  m->symmetric_alpha_ = opt[6] != 0;
  m->print_log_likelihood_ = opt[7] != 0;
  m->num_threads_ = opt[8];
  m->sampler_ = opt[9];
  const int64_t big = (int64_t)1 << 40;
  m->doc_off_ = r.vec<int64_t>(big);
  m->words_ = r.vec<int32_t>(big);
  m->z_cache_ = r.vec<int32_t>(big);
  const int64_t D = (int64_t)m->doc_off_.size() - 1;
  if (D < 0 || m->doc_off_[0] != 0 || m->doc_off_.back() != (int64_t)m->words_.size() ||
      (!m->z_cache_.empty() && m->z_cache_.size() != m->words_.size()))
    raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (documents)");
  for (int32_t wid : m->words_)
    if (wid < 0 || wid >= V) raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (word id)");
  for (int32_t t : m->z_cache_)
    if (t < 0 || t >= K) raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (topic)");
  const int64_t na = r.count(V);
  for (int64_t i = 0; i < na; ++i) m->alphabet_.push_back(r.str());
  m->has_source_ = r.vec<uint8_t>(D);
  for (int64_t d = 0; d < (int64_t)m->has_source_.size(); ++d) m->sources_.push_back(r.str());
  m->max_doc_len_ = r.pod<int32_t>();
  if (v1 || v2 || v3) {            // the histograms older files carry: read past them
    const std::vector<int32_t> dl = r.vec<int32_t>(big), td = r.vec<int32_t>(big);
    if (m->max_doc_len_ >= 0 &&
        (dl.size() != (size_t)m->max_doc_len_ + 1 || td.size() != (size_t)K * (m->max_doc_len_ + 1)))
      raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (statistics)");
  }
  if ((int64_t)m->has_source_.size() != D) raise(LDA_ERR_INVALID_ARG, "checkpoint corrupt (sources)");
  if (m->max_doc_len_ >= 0) {
    m->doc_len_counts_.assign((size_t)m->max_doc_len_ + 1, 0);
    m->topic_doc_counts_.assign((size_t)K * (m->max_doc_len_ + 1), 0);
  }
  if (!v1) {
    m->warm_parts_ = r.pod<int32_t>();
    m->warm_sweeps_ = r.pod<int32_t>();
  }
  // files before v3 continue with the snapshot sweeps they were made with
  m->staleness_threads_ = (v1 || v2) ? -1 : r.pod<int32_t>();
  m->shards_dirty_ = true;
  return m;
}

void ParallelTopicModel::infer(int64_t Dh, const int64_t* doc_off, const int32_t* words,
                               int32_t num_iterations, int32_t thinning, int32_t burn_in,
                               uint64_t seed, double* theta) {
  ensureShards();
  if (Dh < 0 || (Dh > 0 && (!doc_off || !theta))) raise(LDA_ERR_INVALID_ARG, "bad documents");
  // tokens of types unknown to the model are dropped (Mallet's inferencer
  // skips type indices beyond its typeTopicCounts); lda_infer also skips
  // known types without training tokens
  std::vector<int64_t> off((size_t)Dh + 1, 0);
  std::vector<int32_t> kept;
  for (int64_t d = 0; d < Dh; ++d) {
    for (int64_t i = doc_off[d] - doc_off[0]; i < doc_off[d + 1] - doc_off[0]; ++i)
      if (words[i] >= 0 && words[i] < V_) kept.push_back(words[i]);
    off[(size_t)d + 1] = (int64_t)kept.size();
  }
  check(lda_infer(shards_->ctx[0], Dh, off.data(), kept.empty() ? nullptr : kept.data(),
                  num_iterations, thinning, burn_in, seed, theta),
        "lda_infer");
}

}  // namespace lda_host

// ------------------------------------------------------------------ C ABI
struct ldatm {
  std::unique_ptr<lda_host::ParallelTopicModel> owned;
  lda_host::ParallelTopicModel& model;
  ldatm(int32_t K, double a, double b)
      : owned(std::make_unique<lda_host::ParallelTopicModel>(K, a, b)), model(*owned) {}
  explicit ldatm(std::unique_ptr<lda_host::ParallelTopicModel> m) : owned(std::move(m)), model(*owned) {}
};

namespace {
thread_local std::string g_tm_error;

template <typename F>
lda_status guard(F&& f) {
  try {
    f();
    return LDA_OK;
  } catch (const lda_host::Error& e) {
    g_tm_error = e.message;
    return e.status;
  } catch (const std::bad_alloc&) {
    g_tm_error = "host allocation failed";
    return LDA_ERR_OUT_OF_MEMORY;
  } catch (const std::exception& e) {
    g_tm_error = e.what();
    return LDA_ERR_INVALID_ARG;
  } catch (...) {
    g_tm_error = "internal error: unknown exception";
    return LDA_ERR_INTERNAL;
  }
}

lda_status copy_text(const std::string& s, char* buf, size_t cap, size_t* len) {
  if (len) *len = s.size();
  if (buf) {
    if (cap < s.size() + 1) {
      g_tm_error = "buffer too small";
      return LDA_ERR_INVALID_ARG;
    }
    std::memcpy(buf, s.c_str(), s.size() + 1);
  }
  return LDA_OK;
}

lda_status write_file(const char* path, const std::string& s) {
  if (!path) {
    g_tm_error = "null path";
    return LDA_ERR_INVALID_ARG;
  }
  bool ok = false;
  const lda_status st = guard([&] {
    std::ofstream f(path, std::ios::binary);
    if (!f) throw lda_host::Error{LDA_ERR_INVALID_ARG, std::string("cannot open ") + path};
    f << s;
    ok = f.good();
  });
  if (st) return st;
  if (!ok) g_tm_error = std::string("write failed: ") + path;
  return ok ? LDA_OK : LDA_ERR_INVALID_ARG;
}

#define TM_CHECK(m)                 \
  if (!(m)) {                       \
    g_tm_error = "null model";      \
    return LDA_ERR_INVALID_ARG;     \
  }
}  // namespace

extern "C" {

const char* ldatm_last_error(void) { return g_tm_error.c_str(); }

lda_status ldatm_format_double(double x, int32_t style, char* buf, size_t cap) {
  if (style != 0 && style != 1) {
    g_tm_error = "style must be 0 or 1";
    return LDA_ERR_INVALID_ARG;
  }
  std::string t;
  const lda_status st = guard([&] { t = style == 0 ? lda_host::java_double(x) : lda_host::java_number5(x); });
  return st ? st : copy_text(t, buf, cap, nullptr);
}

lda_status ldatm_create(ldatm** out, int32_t num_topics, double alpha_sum, double beta) {
  if (!out) return LDA_ERR_INVALID_ARG;
  *out = nullptr;
  return guard([&] { *out = new ldatm(num_topics, alpha_sum, beta); });
}

void ldatm_destroy(ldatm* m) { delete m; }

lda_status ldatm_set_alphabet(ldatm* m, int32_t num_types, const char* const* words) {
  TM_CHECK(m);
  return guard([&] {
    std::vector<std::string> w;
    if (words)
      for (int32_t i = 0; i < num_types; ++i) w.emplace_back(words[i] ? words[i] : "");
    m->model.setAlphabet(std::move(w), num_types);
  });
}

lda_status ldatm_add_instances(ldatm* m, int64_t D, const int64_t* doc_off, const int32_t* words,
                               const char* const* sources) {
  TM_CHECK(m);
  return guard([&] { m->model.addInstances(D, doc_off, words, sources); });
}

#define TM_SETTER(name, call)                          \
  lda_status name(ldatm* m, int32_t n) {               \
    TM_CHECK(m);                                       \
    return guard([&] { m->model.call; });              \
  }
TM_SETTER(ldatm_set_num_iterations, setNumIterations(n))
TM_SETTER(ldatm_set_optimize_interval, setOptimizeInterval(n))
TM_SETTER(ldatm_set_burnin_period, setBurninPeriod(n))
TM_SETTER(ldatm_set_symmetric_alpha, setSymmetricAlpha(n != 0))
TM_SETTER(ldatm_set_num_threads, setNumThreads(n))
TM_SETTER(ldatm_set_sampler, setSampler(n))
TM_SETTER(ldatm_set_exchange_parts, setExchangeParts(n))

lda_status ldatm_set_warm_start(ldatm* m, int32_t parts, int32_t sweeps) {
  TM_CHECK(m);
  return guard([&] { m->model.setWarmStart(parts, sweeps); });
}

lda_status ldatm_set_staleness_threads(ldatm* m, int32_t threads) {
  TM_CHECK(m);
  return guard([&] { m->model.setStalenessThreads(threads); });
}

lda_status ldatm_set_devices(ldatm* m, int32_t n, const int32_t* devices) {
  TM_CHECK(m);
  return guard([&] { m->model.setDevices(devices, n); });
}

lda_status ldatm_num_shards(ldatm* m, int32_t* shards) {
  TM_CHECK(m && shards);
  return guard([&] { *shards = m->model.numShards(); });
}

lda_status ldatm_exchange_info(ldatm* m, int32_t* cells_per_word, int32_t* used_lists, int32_t* escapes_max,
                               int64_t* list_exchanges) {
  TM_CHECK(m);
  return guard([&] { m->model.exchangeInfo(cells_per_word, used_lists, escapes_max, list_exchanges); });
}

int32_t ldatm_plan_shards(int32_t num_threads, int32_t num_devices, int64_t num_tokens,
                          int32_t num_types, int32_t num_topics, int64_t num_docs) {
  return lda_host::plan_shards(num_threads, num_devices, num_tokens, num_types, num_topics, num_docs);
}
TM_SETTER(ldatm_set_verbosity, setVerbosity(n))
TM_SETTER(ldatm_set_print_log_likelihood, setPrintLogLikelihood(n != 0))

lda_status ldatm_set_save_sample_interval(ldatm* m, int32_t n) {
  TM_CHECK(m);
  if (n < 1) {
    g_tm_error = "saveSampleInterval must be >= 1";
    return LDA_ERR_INVALID_ARG;
  }
  return guard([&] { m->model.setSaveSampleInterval(n); });
}

lda_status ldatm_set_topic_display(ldatm* m, int32_t interval, int32_t n) {
  TM_CHECK(m);
  return guard([&] { m->model.setTopicDisplay(interval, n); });
}

lda_status ldatm_set_random_seed(ldatm* m, int64_t seed) {
  TM_CHECK(m);
  return guard([&] { m->model.setRandomSeed(seed); });
}

lda_status ldatm_set_topics(ldatm* m, int64_t n, const int32_t* z) {
  TM_CHECK(m);
  TM_CHECK(z || n == 0);
  return guard([&] { m->model.setTopics(z, n); });
}

lda_status ldatm_set_hyper(ldatm* m, const double* alpha, double alpha_sum, double beta) {
  TM_CHECK(m && alpha);
  return guard([&] { m->model.setHyper(alpha, alpha_sum, beta); });
}

lda_status ldatm_get_sweep(ldatm* m, uint32_t* sweep) {
  TM_CHECK(m && sweep);
  return guard([&] { *sweep = m->model.sweep(); });
}

lda_status ldatm_set_sweep(ldatm* m, uint32_t sweep) {
  TM_CHECK(m);
  return guard([&] { m->model.setSweep(sweep); });
}

lda_status ldatm_estimate(ldatm* m) {
  TM_CHECK(m);
  return guard([&] { m->model.estimate(); });
}

lda_status ldatm_get_ll_trace(ldatm* m, int32_t* iterations, double* ll, int32_t cap, int32_t* n) {
  TM_CHECK(m);
  const auto& t = m->model.llTrace();
  if (n) *n = (int32_t)t.size();
  for (int32_t i = 0; i < cap && i < (int32_t)t.size(); ++i) {
    if (iterations) iterations[i] = t[(size_t)i].first;
    if (ll) ll[i] = t[(size_t)i].second;
  }
  return LDA_OK;
}

lda_status ldatm_model_log_likelihood(ldatm* m, double* out) {
  TM_CHECK(m);
  return guard([&] { *out = m->model.modelLogLikelihood(); });
}

lda_status ldatm_get_shape(ldatm* m, int32_t* K, int32_t* V, int64_t* D, int64_t* N) {
  TM_CHECK(m);
  if (K) *K = m->model.numTopics();
  if (V) *V = m->model.numTypes();
  if (D) *D = m->model.numDocs();
  if (N) *N = m->model.numTokens();
  return LDA_OK;
}

lda_status ldatm_get_hyper(ldatm* m, double* alpha, double* alpha_sum, double* beta) {
  TM_CHECK(m);
  if (alpha) std::copy(m->model.alpha().begin(), m->model.alpha().end(), alpha);
  if (alpha_sum) *alpha_sum = m->model.alphaSum();
  if (beta) *beta = m->model.beta();
  return LDA_OK;
}

lda_status ldatm_get_z(ldatm* m, int32_t* z) {
  TM_CHECK(m);
  return guard([&] {
    const std::vector<int32_t> t = m->model.topics();
    if ((int64_t)t.size() != m->model.numTokens()) throw lda_host::Error{LDA_ERR_STATE, "no topic assignments yet"};
    std::copy(t.begin(), t.end(), z);
  });
}

lda_status ldatm_get_counts(ldatm* m, int32_t* nw, int32_t* nwsum) {
  TM_CHECK(m);
  return guard([&] { m->model.counts(nw, nwsum); });
}

lda_status ldatm_get_topic_probabilities(ldatm* m, int64_t doc, double* out) {
  TM_CHECK(m);
  return guard([&] {
    const std::vector<double> p = m->model.getTopicProbabilities(doc);
    std::copy(p.begin(), p.end(), out);
  });
}

lda_status ldatm_document_topics_text(ldatm* m, double threshold, int32_t max, char* buf, size_t cap,
                                      size_t* len) {
  TM_CHECK(m);
  std::string s;
  lda_status st = guard([&] { s = m->model.documentTopics(threshold, max); });
  return st ? st : copy_text(s, buf, cap, len);
}

lda_status ldatm_print_document_topics(ldatm* m, const char* path, double threshold, int32_t max) {
  TM_CHECK(m);
  std::string s;
  lda_status st = guard([&] { s = m->model.documentTopics(threshold, max); });
  return st ? st : write_file(path, s);
}

lda_status ldatm_top_words_text(ldatm* m, int32_t num_words, int32_t using_new_lines, char* buf,
                                size_t cap, size_t* len) {
  TM_CHECK(m);
  std::string s;
  lda_status st = guard([&] { s = m->model.displayTopWords(num_words, using_new_lines != 0); });
  return st ? st : copy_text(s, buf, cap, len);
}

lda_status ldatm_print_top_words(ldatm* m, const char* path, int32_t num_words, int32_t using_new_lines) {
  TM_CHECK(m);
  std::string s;
  lda_status st = guard([&] { s = m->model.displayTopWords(num_words, using_new_lines != 0); });
  return st ? st : write_file(path, s);
}

lda_status ldatm_save(ldatm* m, const char* path) {
  TM_CHECK(m);
  if (!path) {
    g_tm_error = "null path";
    return LDA_ERR_INVALID_ARG;
  }
  return guard([&] { m->model.save(path); });
}

lda_status ldatm_load(ldatm** out, const char* path) {
  if (!out || !path) {
    g_tm_error = "null argument";
    return LDA_ERR_INVALID_ARG;
  }
  *out = nullptr;
  return guard([&] {
    auto loaded = lda_host::ParallelTopicModel::load(path);
    *out = new ldatm(std::move(loaded));
  });
}

lda_status ldatm_infer(ldatm* m, int64_t Dh, const int64_t* doc_off, const int32_t* words,
                       int32_t num_iterations, int32_t thinning, int32_t burn_in, uint64_t seed,
                       double* theta) {
  TM_CHECK(m);
  return guard([&] { m->model.infer(Dh, doc_off, words, num_iterations, thinning, burn_in, seed, theta); });
}

}  // extern "C"
