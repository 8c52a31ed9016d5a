// lda_kernels.hip — gfx950 (MI355X / CDNA4) kernels of the collapsed-Gibbs
// LDA sampler.  Replaces the per-token loop of Mallet 2.0.7's
// WorkerRunnable.sampleTopicsForOneDoc, reached from ParallelTopicModel.
// estimate() at src/cmu_ron/TrainAndPredict.java:166 and
// src/cmu/TrainAndPredict.java:265 of the reference.
//
// Sampling semantics: AD-LDA with a per-sweep
// snapshot.  nw/nwsum are read-only during a pass (the token's own old
// assignment is subtracted on the fly), nd is live inside a document, and all
// count changes go to an int32 delta buffer that lda_apply folds in after the
// pass (after an RCCL all-reduce when the corpus is sharded over GPUs).
// Integer adds commute, so z/nw/nwsum are independent of scheduling, of the
// number of GPUs, and bit-identical to the CPU oracle (oracle/lda_oracle.c).
//
// Exact fp32 evaluation order of one draw (mirrored by oracle exact_draw):
//   lane l owns topics [l*C, l*C+C), C = Kp/64.
//   b_k  = (float(nw_wk - [k==zo]) + beta) * (k==zo ? inv_m1_k : inv_k)
//   a_k  = float(nd_k) + alpha_k
//   S_j  = fma(a_j, b_j, S_{j-1}), S_{-1} = 0   (serial inside the lane)
//   T    = wave_incl_scan(S_{C-1})              (DPP order, see below)
//   thr  = u * T_63,  u = (x0 >> 8) * 2^-24, x0 = Philox4x32-10 word 0
//   l*   = first lane <= last_lane with T_l > thr, else last_lane
//   j*   = #{j : T_{l*-1} + S_j <= thr} (S is monotone) or, if that is C,
//          the last valid topic of lane l*
//   z    = l*·C + j*
//
// Compiled with -ffp-contract=off: the only fused multiply-adds are the
// explicit __builtin_fmaf below.
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "lda_kernels.h"

namespace lda {

// ---------------------------------------------------------------- Philox
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

__device__ __forceinline__ uint32_t philox_x0(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += PHILOX_W0;
      k1 += PHILOX_W1;
    }
    const uint32_t hi0 = __umulhi(PHILOX_M0, c0), lo0 = PHILOX_M0 * c0;
    const uint32_t hi1 = __umulhi(PHILOX_M1, c2), lo1 = PHILOX_M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  return c0;
}

__device__ __forceinline__ uint32_t draw_u32(uint64_t gtok, uint32_t c2, uint32_t c3, uint32_t k0,
                                             uint32_t k1) {
  return philox_x0((uint32_t)gtok, (uint32_t)(gtok >> 32), c2, c3, k0, k1);
}

__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * 0x1p-24f; }

// ------------------------------------------------------------ wave helpers
template <int CTRL, int ROW_MASK, bool BOUND>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(
      float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, BOUND));
}

// Inclusive wavefront scan: row_shr:1,2,4,8 inside 16-lane rows (sources
// outside the row read 0), row_bcast:15 into rows 1 and 3, row_bcast:31 into
// rows 2 and 3.  Restated lane by lane in oracle/lda_oracle.c:wave_scan_emulate.
#ifndef LDA_ASM_SCAN
#define LDA_ASM_SCAN 1
#endif
#ifndef LDA_GPRIDX
#define LDA_GPRIDX 1
#endif
#ifndef LDA_UPD_MASK
#define LDA_UPD_MASK 1
#endif
#ifndef LDA_SALU_TRIM
#define LDA_SALU_TRIM 1
#endif
// Keep the row prefetch a real pipeline: vmcnt counts vector memory
// operations in issue order, and the compiler waits for row t while row t+1
// stays in flight (vmcnt(P-1)) only when every token issues the same number
// of them.  So the delta atomics are issued per 64-token chunk instead of per
// token (LDA_CHUNK_DELTA), the prefetch load is unconditional, and the rare
// int32-row load drains itself (LDA_WIDE_DRAIN).  Without them every token
// waited vmcnt(0), i.e. for the row prefetched one token earlier.
#ifndef LDA_WIDE_DRAIN
#define LDA_WIDE_DRAIN 1
#endif
#ifndef LDA_CHUNK_DELTA
#define LDA_CHUNK_DELTA 1
#endif
#ifndef LDA_SALU_COUNT
#define LDA_SALU_COUNT 1
#endif
#ifndef LDA_WORD_FLAG
#define LDA_WORD_FLAG 1
#endif
// s_waitcnt vmcnt(0) / vmcnt(1) (gfx9 encoding: expcnt and lgkmcnt left at their maxima)
constexpr int kVmcnt0 = 0x0F70;
constexpr int kVmcnt1 = 0x0F71;
constexpr int kLgkmcnt0 = 0xC07F;   // lgkmcnt(0), vmcnt and expcnt left at their maxima
// (a != b) ? m : 0 as s_cmp + s_cselect_b64
__device__ __forceinline__ uint64_t select_mask_ne(int a, int b, uint64_t m) {
  uint64_t r;
  // the operands are wave-uniform; readfirstlane keeps them in SGPRs even
  // where the compiler's divergence analysis cannot tell
  a = __builtin_amdgcn_readfirstlane(a);
  b = __builtin_amdgcn_readfirstlane(b);
  asm("s_cmp_lg_u32 %1, %2\n\ts_cselect_b64 %0, %3, 0" : "=s"(r) : "s"(a), "s"(b), "s"(m) : "scc");
  return r;
}
// (jo == J) ? m : 0 for J = 0..C-1 (immediate J: no constant in an SGPR)
template <int J>
__device__ __forceinline__ uint64_t select_mask_c(int jo, uint64_t m) {
  uint64_t r;
  jo = __builtin_amdgcn_readfirstlane(jo);
  asm("s_cmp_eq_u32 %1, %2\n\ts_cselect_b64 %0, %3, 0" : "=s"(r) : "s"(jo), "n"(J), "s"(m) : "scc");
  return r;
}
template <int C, int J = 0>
__device__ __forceinline__ void fill_masks(uint64_t (&jm)[C], int jo, uint64_t m) {
  if constexpr (J < C) {
    jm[J] = select_mask_c<J>(jo, m);
    fill_masks<C, J + 1>(jm, jo, m);
  }
}
// the lowest set lane of m, or `none` when m is empty (s_ff1 gives -1 for 0)
__device__ __forceinline__ int first_lane_or(uint64_t m, int none) {
  int r;
  none = __builtin_amdgcn_readfirstlane(none);
  asm("s_ff1_i32_b64 %0, %1\n\ts_min_u32 %0, %0, %2" : "=&s"(r) : "s"(m), "s"(none) : "scc");
  return r;
}
// (jo == j) ? m : 0 as s_cmp + s_cselect_b64 (the compiler splits the 64-bit
// select in two and adds an s_and)
__device__ __forceinline__ uint64_t select_mask(int jo, int j, uint64_t m) {
  uint64_t r;
  jo = __builtin_amdgcn_readfirstlane(jo);
  asm("s_cmp_eq_u32 %1, %2\n\ts_cselect_b64 %0, %3, 0" : "=s"(r) : "s"(jo), "s"(j), "s"(m) : "scc");
  return r;
}
// c + bit l of m (s_bitcmp1_b64 sets SCC, s_addc_u32 adds it)
__device__ __forceinline__ int add_lane_bit(int c, uint64_t m, int l) {
  l = __builtin_amdgcn_readfirstlane(l);
  c = __builtin_amdgcn_readfirstlane(c);
  asm("s_bitcmp1_b64 %1, %2\n\ts_addc_u32 %0, %0, 0" : "+s"(c) : "s"(m), "s"(l) : "scc");
  return c;
}
__device__ __forceinline__ float wave_incl_scan(float x) {
  x = dpp_mov<0x111, 0xf, true>(x) + x;
  x = dpp_mov<0x112, 0xf, true>(x) + x;
  x = dpp_mov<0x114, 0xf, true>(x) + x;
  x = dpp_mov<0x118, 0xf, true>(x) + x;
#if LDA_ASM_SCAN
  // The two broadcast steps as one masked DPP add each: rows outside the row
  // mask are not written and keep x (= x + 0 of the two-instruction form).
  // s_nop 1: a VALU-written VGPR needs two wait states before a DPP read.
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(x));
#else
  x = x + dpp_mov<0x142, 0xa, false>(x);
  x = x + dpp_mov<0x143, 0xc, false>(x);
#endif
  return x;
}

__device__ __forceinline__ int readlane_i(int v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ float readlane_f(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ int uniform_i(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uniform_l(int64_t v) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(v >> 32)) << 32) |
                   (uint32_t)__builtin_amdgcn_readfirstlane((int)v));
}

// Lanes of one wavefront hand LDS values to each other (histogram atomics,
// lane-0 updates read by every lane).  Without a fence that is a data race in
// the C++ model and hipcc may forward a lane's OWN earlier store to its later
// load (observed: the doc-histogram zeroing store forwarded past other lanes'
// ds_add).  A wavefront-scope fence is a compiler memory barrier; DS
// instructions of one wave already execute in order, so it costs nothing.
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

// The next work range of a consumer (a wave, or a 16-lane row of the
// quarter-wave kernel): its first is static -- consumer `id` of `count`
// takes range id -- and later ones come from the queue, offset by count.
// A launch's first grab was a burst of same-address atomics from every
// consumer at once; a small corpus (C1: ~1000 ranges, one per wave) now
// takes none.  Which consumer samples which range never changes a result
// (draws are keyed by the global token index).  The wave kernels pass the
// result through uniform_i: the id derives from threadIdx.x, which the
// compiler cannot tell is wave-uniform, and every branch on the range's
// bounds downstream of it had become an exec-mask branch (scalar work).
#ifndef LDA_STATIC_FIRST
#define LDA_STATIC_FIRST 1
#endif
__device__ __forceinline__ int first_or_queued(bool first, int id, int count, int queued) {
  return (LDA_STATIC_FIRST && first) ? id : (LDA_STATIC_FIRST ? count : 0) + queued;
}

template <int C>
__device__ __forceinline__ void load_row(int32_t (&r)[C], const int32_t* __restrict__ p) {
  if constexpr (C >= 4) {
#pragma unroll
    for (int q = 0; q < C / 4; ++q) {
      const int4 v = reinterpret_cast<const int4*>(p)[q];
      r[4 * q + 0] = v.x;
      r[4 * q + 1] = v.y;
      r[4 * q + 2] = v.z;
      r[4 * q + 3] = v.w;
    }
  } else if constexpr (C == 2) {
    const int2 v = *reinterpret_cast<const int2*>(p);
    r[0] = v.x;
    r[1] = v.y;
  } else {
    r[0] = p[0];
  }
}

// ------------------------------------------------------------- the sampler
// One wavefront walks one work range (a run of whole documents) at a time,
// pulling ranges from a device queue.  The wave keeps a 64-token chunk of the
// token stream in registers (lane i <-> token i of the chunk: word, old z,
// Philox uniform, new z), the next two chunks' words/z ahead of it, and the
// 16-bit rows of nw for the next P tokens in flight (the snapshot makes them
// independent of the draws, so they pipeline across tokens and documents).
// Per lane and topic the draw is one fma:
//   S_j = fma(a_j, b_j, S_{j-1}),  a_j = float(nd_j) + alpha_j (LDS, per wave)
//   b_j = (float(c_j) + beta) * inv_j  (c_j from the row; packed fp32 pairs)
// and the z_old element of lane z_old/C uses the own-token-corrected factor
// ((float)(c_zold - 1) + beta) * inv_m1[z_old], c_zold taken from the row.

template <int C>
__device__ __forceinline__ void load_lds_f(float (&r)[C], const float* p) {
  if constexpr (C >= 4) {
#pragma unroll
    for (int q = 0; q < C / 4; ++q) {
      const float4 v = reinterpret_cast<const float4*>(p)[q];
      r[4 * q + 0] = v.x;
      r[4 * q + 1] = v.y;
      r[4 * q + 2] = v.z;
      r[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < C; ++j) r[j] = p[j];
  }
}

// Row of 16-bit counts: C u16 per lane = C/2 dwords (C >= 2), one u16 for C = 1.
template <int C>
__device__ __forceinline__ void load_row16(uint32_t (&r)[(C + 1) / 2], const uint16_t* __restrict__ row,
                                           int lane) {
  if constexpr (C >= 8) {
#pragma unroll
    for (int q = 0; q < C / 8; ++q) {
      const uint4 v = reinterpret_cast<const uint4*>(row + lane * C)[q];
      r[4 * q + 0] = v.x;
      r[4 * q + 1] = v.y;
      r[4 * q + 2] = v.z;
      r[4 * q + 3] = v.w;
    }
  } else if constexpr (C == 4) {
    const uint2 v = *reinterpret_cast<const uint2*>(row + lane * C);
    r[0] = v.x;
    r[1] = v.y;
  } else if constexpr (C == 2) {
    r[0] = *reinterpret_cast<const uint32_t*>(row + lane * C);
  } else {
    r[0] = row[lane];
  }
}

template <int C>
__device__ __forceinline__ int32_t row16_count(const uint32_t (&r)[(C + 1) / 2], int j) {
  if constexpr (C == 1) return (int32_t)r[0];
  else return (int32_t)((j & 1) ? (r[j >> 1] >> 16) : (r[j >> 1] & 0xFFFFu));
}

typedef float pkf32 __attribute__((ext_vector_type(2)));

// Minimum waves per SIMD the compiler must fit the dense sampler into (a few
// spilled registers are cheaper than a lost wave: A/B on C4 at C = 8, 7 waves
// with 5 spills vs 6 without is +6%).  SAMPLE_WPE_C<C> overrides for A/B runs.
template <int C>
constexpr int sample_waves_per_eu() {
#if defined(SAMPLE_WPE_C1)
  if (C == 1) return SAMPLE_WPE_C1;
#endif
#if defined(SAMPLE_WPE_C2)
  if (C == 2) return SAMPLE_WPE_C2;
#endif
#if defined(SAMPLE_WPE_C4)
  if (C == 4) return SAMPLE_WPE_C4;
#endif
#if defined(SAMPLE_WPE_C8)
  if (C == 8) return SAMPLE_WPE_C8;
#endif
#if defined(SAMPLE_WPE_C16)
  if (C == 16) return SAMPLE_WPE_C16;
#endif
  return C == 8 ? 7 : 1;
}

// Lane i gets a[i + S] for i + S < 64, else b[i + S - 64] (a wave-wide
// shift across two chunk registers; two ds_bpermutes).
template <int S>
__device__ __forceinline__ int shift_in(int a, int b, int lane) {
  const int src = (lane + S) & 63;
  const int va = __shfl(a, src), vb = __shfl(b, src);
  return lane + S < 64 ? va : vb;
}

template <int C, int P, bool FROZEN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(sample_waves_per_eu<C>())))
void k_sample(SampleParams p) {
  if (p.state_dev) {                                  // a graph-launched sweep (lda_sweep)
    p.c2 = p.state_dev[0];
    p.beta = __uint_as_float(p.state_dev[1]);
  }
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  constexpr int KP = C * 64;
  constexpr int H = (C + 1) / 2;                     // dwords of a 16-bit row per lane
  // inv_m1 as a per-block LDS table for C <= 8; for C = 16 the extra table
  // would cost a block per CU, so inv_m1[z_old] is prefetched from memory
  constexpr bool kInvLds = C <= 8;
  constexpr bool kInvM1Lds = kInvLds;
  constexpr int TB = kInvLds ? 3 : 2;                // per-block tables before the per-wave area
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float* t_alpha = reinterpret_cast<float*>(smem);   // [KP] per block
  int32_t* bsum = smem + KP;                         // [KP] per-block nwsum delta
  float* t_invm1 = reinterpret_cast<float*>(smem + 2 * KP);  // [KP] per block (kInvLds)
  int32_t* nd = smem + TB * KP + wid * 2 * KP;       // [KP] per-wave live doc counts
  float* av = reinterpret_cast<float*>(nd + KP);     // [KP] per-wave a_k = float(nd_k) + alpha_k

  for (int i = threadIdx.x; i < KP; i += 256) {
    t_alpha[i] = p.alpha[i];
    bsum[i] = 0;
    if (kInvM1Lds) t_invm1[i] = FROZEN ? 0.0f : p.inv_m1[i];
  }
  for (int i = threadIdx.x; i < 8 * KP; i += 256) smem[TB * KP + i] = 0;
  __syncthreads();

  float inv_r[C];
#pragma unroll
  for (int j = 0; j < C; ++j) inv_r[j] = p.inv[lane * C + j];
  const float beta = p.beta;
  const uint64_t lt2_mask = __ballot(lane < 2);
  const int last_lane = (p.K - 1) / C;
  const uint64_t last_mask = __ballot(lane <= last_lane);
  const int last_j_tail = (p.K - 1) % C;
  const uint16_t* __restrict__ nw16 = p.nw16;
  const uint8_t* __restrict__ wide_of = p.wide;
  const int32_t* __restrict__ nw = p.nw;
  const float* __restrict__ inv_m1 = p.inv_m1;

  bool first_range = true;
  while (true) {
    int r = 0;
    if ((!LDA_STATIC_FIRST || !first_range) && lane == 0) r = atomicAdd(p.queue, 1);
    r = uniform_i(first_or_queued(first_range, (int)blockIdx.x * 4 + wid, (int)gridDim.x * 4, uniform_i(__shfl(r, 0))));
    first_range = false;
    if (r >= p.num_ranges) break;
    const int64_t d0 = p.range_doc[r], d1 = p.range_end[r];
    const int64_t t0 = p.doc_off[d0];
    // token positions below are 32-bit offsets from the range start
    const int nt = (int)(p.doc_off[d1] - t0);
    if (nt <= 0) continue;
    const int32_t* __restrict__ wrd = p.words + t0;
    int32_t* __restrict__ zr = p.z + t0;
    const uint64_t gbase = (uint64_t)(p.token_base + t0);
    // a finished chunk's count changes, lane i = token cbase + i (word w_,
    // topic zo_ -> zn_): two wave-wide atomics per 64 tokens; the 32-bit cell
    // index is valid because lda_create keeps V*Kp < 2^32
    auto flush_delta = [&](int w_, int zo_, int zn_) {
      if (!FROZEN && LDA_CHUNK_DELTA && p.delta && zn_ != zo_) {
        const uint32_t row = (uint32_t)w_ * (uint32_t)KP;
        atomicAdd(p.delta + (row + (uint32_t)zo_), -1);
        atomicAdd(p.delta + (row + (uint32_t)zn_), 1);
        atomicAdd(&bsum[zo_], -1);
        atomicAdd(&bsum[zn_], 1);
      }
    };

    // --- chunk registers: chunk c (cw, cz, cu, cn, cf), c+1 (w1, z1, f1), c+2 (w2, z2);
    // f = 1 when the word's row holds a count > 65535 (read the int32 row)
    int cbase = 0;
    int cw = 0, cz = 0, w1 = 0, z1 = 0, w2 = 0, z2 = 0;
    if (lane < nt) {
      cw = wrd[lane];
      cz = zr[lane];
    }
    if (64 + lane < nt) {
      w1 = wrd[64 + lane];
      z1 = zr[64 + lane];
    }
    if (128 + lane < nt) {
      w2 = wrd[128 + lane];
      z2 = zr[128 + lane];
    }
    // kWordFlag: the int32-row flag rides in bit 31 of the word registers
    // (one readlane per token for both; word ids are < 2^31)
    constexpr bool kWordFlag = LDA_WORD_FLAG;
    constexpr int kWordMask = 0x7FFFFFFF;
    int cf = 0, f1 = 0;
    if constexpr (kWordFlag) {
      cw |= (int)wide_of[cw] << 31;
      w1 |= (int)wide_of[w1] << 31;
    } else {
      cf = (int)wide_of[cw];
      f1 = (int)wide_of[w1];
    }
    int cn = cz;
    float cu = u01(draw_u32(gbase + (uint64_t)lane, p.c2, p.c3, p.k0, p.k1));
    // word (and, for the inv_m1 prefetch, topic) of token cbase + lane + P:
    // the row prefetch reads it with one readlane instead of branching
    // between chunks
    int pw = shift_in<P>(cw, w1, lane);
    int pz = kInvM1Lds ? 0 : shift_in<P>(cz, z1, lane);

    // --- first document of the range (nd is all zero here)
    int64_t doc = d0;
    while (p.doc_off[doc + 1] <= t0) ++doc;
    int doc_end = uniform_i((int)(p.doc_off[doc + 1] - t0));
    {
      for (int i = lane; i < doc_end; i += 64) atomicAdd(&nd[zr[i]], 1);
      wave_lds_fence();
#pragma unroll
      for (int j = 0; j < C; ++j) av[lane * C + j] = (float)nd[lane * C + j] + t_alpha[lane * C + j];
      wave_lds_fence();
    }

    int kp = 0, inc = 0;              // deferred add-back of the last drawn token
    int ev = min(64, doc_end);        // token index of the next chunk or document start

    // --- prime the pipeline: 16-bit rows of the next P tokens
    uint32_t rows[P][H];
    float cinv_r[P];
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const int wp = (s < nt) ? (readlane_i(cw, s) & kWordMask) : 0;
      load_row16<C>(rows[s], nw16 + (int64_t)wp * KP, lane);
      if (!FROZEN && !kInvM1Lds) cinv_r[s] = inv_m1[(s < nt) ? readlane_i(cz, s) : 0];
    }

    // one token (slot s of its group of P: rows[s] holds its row)
    auto token = [&](const int t, const int s) __attribute__((always_inline)) {
        if (t == ev) {
          // the next chunk and/or the next document start here (one compare
          // per token for both)
          if (t - cbase == 64) {
            // chunk switch: publish the finished chunk's new z and count
            // changes, shift
            zr[cbase + lane] = cn;
            flush_delta(cw & kWordMask, cz, cn);
            cbase += 64;
            cw = w1;
            cz = z1;
            cf = f1;
            w1 = w2;
            z1 = z2;
            if constexpr (kWordFlag) w1 |= (int)wide_of[w1] << 31;
            else f1 = (int)wide_of[w1];
            cn = cz;
            cu = u01(draw_u32(gbase + (uint64_t)(cbase + lane), p.c2, p.c3, p.k0, p.k1));
            if (cbase + 128 + lane < nt) {
              w2 = wrd[cbase + 128 + lane];
              z2 = zr[cbase + 128 + lane];
            }
            pw = shift_in<P>(cw, w1, lane);
            if constexpr (!kInvM1Lds) pz = shift_in<P>(cz, z1, lane);
          }
          if (t == doc_end) {
            inc = 0;                  // the pending add belonged to the last document
#pragma unroll
            for (int j = 0; j < C; ++j) nd[lane * C + j] = 0;
            wave_lds_fence();
            ++doc;
            while (p.doc_off[doc + 1] - t0 <= t) ++doc;
            doc_end = uniform_i((int)(p.doc_off[doc + 1] - t0));
            for (int i = t + lane; i < doc_end; i += 64) atomicAdd(&nd[zr[i]], 1);
            wave_lds_fence();
#pragma unroll
            for (int j = 0; j < C; ++j) av[lane * C + j] = (float)nd[lane * C + j] + t_alpha[lane * C + j];
            wave_lds_fence();
          }
          ev = min(cbase + 64, doc_end);
        }
        const int idx = t - cbase;

        const int wf = readlane_i(cw, idx);
        const int w = wf & kWordMask;
        const int zo = readlane_i(cz, idx);
        const float u = readlane_f(cu, idx);
        const bool wide = kWordFlag ? wf < 0 : readlane_i(cf, idx) != 0;
#if LDA_SALU_TRIM
        const int lo = (int)((uint32_t)zo / C), jo = (int)((uint32_t)zo % C);
#else
        const int lo = zo / C, jo = zo % C;
#endif

        // lane 0: add the previous token back under its new topic kp (deferred
        // from its draw; inc = 0 at a document's first token), then remove
        // this token from its document
        if (lane == 0) {
          const int ndk = nd[kp] + inc;
          nd[kp] = ndk;
          av[kp] = (float)ndk + t_alpha[kp];
          const int ndz = nd[zo] - 1;
          nd[zo] = ndz;
          av[zo] = (float)ndz + t_alpha[zo];
        }
        wave_lds_fence();
        float a[C];
        load_lds_f<C>(a, av + lane * C);
        const float cinv = FROZEN ? 0.0f : (kInvM1Lds ? t_invm1[zo] : cinv_r[s]);
        // lane lo as a scalar lane mask (s_lshl_b64), selected by inverse ballot
        const uint64_t own_bit = 1ull << (uint32_t)__builtin_amdgcn_readfirstlane(lo);
        const bool own_old = __builtin_amdgcn_inverse_ballot_w64(own_bit);

        // word factors b = (float(c) + beta) * inv (packed fp32 pairs, each
        // half an ordinary IEEE add / mul); rows with a count > 65535 come
        // from the int32 row instead (rare: uniform branch, not prefetched)
        // The own-token correction touches one element, j_old of lane l_old
        // (uniform j_old): for C >= 8 the row is a vector that hipcc indexes
        // with s_set_gpr_idx (one move each for reading c_old and patching b)
        // instead of a select per element and a lane mask per element (C4:
        // 5.93 -> 6.26 G tok/s, although the tuples spill 9 more VGPRs).
        constexpr bool kGprIdx = LDA_GPRIDX && C >= 8;
        // C = 8 rows as 9-wide vectors: hipcc expands a dynamic index into
        // selects for up to 8 elements, and indexes 9 or more with
        // s_set_gpr_idx (the 9th register is never addressed: jo < C)
        constexpr int CV = (kGprIdx && C == 8) ? 9 : C;
        typedef int32_t civ __attribute__((ext_vector_type(CV)));
        typedef float cfv __attribute__((ext_vector_type(CV)));
        civ cfull;
        if (wide) {
          const int32_t* wr = nw + (int64_t)w * KP + lane * C;
#pragma unroll
          for (int j = 0; j < C; ++j) cfull[j] = wr[j];
#if LDA_WIDE_DRAIN
          // hipcc lays the 16-bit branch out as a fall-through successor of
          // this block: without this wait, this load in flight into cfull
          // makes it wait vmcnt(0) there too
          __builtin_amdgcn_s_waitcnt(kVmcnt0);
#endif
        } else {
#pragma unroll
          for (int j = 0; j < C; ++j) cfull[j] = row16_count<C>(rows[s], j);
        }
        // the own-token-corrected factor of z_old, from lane lo's own row
        // element (exact: a 16-bit row holds every count below 65536)
        int32_t c_old;
#if LDA_SALU_TRIM
        // one 64-bit lane mask per element: lane lo where j == jo, else none
        // (two SALU ops each; selecting under it is exact on lane lo, the
        // only lane whose value is used)
        const uint64_t own_mask = own_bit;
        uint64_t jmask[kGprIdx ? 1 : C];
        if constexpr (kGprIdx) {
          c_old = cfull[jo];
        } else {
          fill_masks<C>(jmask, jo, own_mask);
          c_old = cfull[0];
#pragma unroll
          for (int j = 1; j < C; ++j) c_old = __builtin_amdgcn_inverse_ballot_w64(jmask[j]) ? cfull[j] : c_old;
        }
#else
        c_old = cfull[0];
#pragma unroll
        for (int j = 1; j < C; ++j) c_old = (j == jo) ? cfull[j] : c_old;
#endif
        const float bc = FROZEN ? 0.0f : ((float)(c_old - 1) + beta) * cinv;
        cfv bw;
        if constexpr (C >= 2) {
#pragma unroll
          for (int j = 0; j < C; j += 2) {
            pkf32 c2v = {(float)cfull[j], (float)cfull[j + 1]};
            const pkf32 b2 = (c2v + beta) * (pkf32){inv_r[j], inv_r[j + 1]};
            bw[j] = b2.x;
            bw[j + 1] = b2.y;
          }
        } else {
          bw[0] = ((float)cfull[0] + beta) * inv_r[0];
        }
        if constexpr (kGprIdx && !FROZEN) {
          const float bo = bw[jo];
          bw[jo] = own_old ? bc : bo;
        }

        // lane-serial fma prefix (the z_old element of lane lo uses bc)
        float S[C];
        float acc = 0.0f;
#pragma unroll
        for (int j = 0; j < C; ++j) {
#if LDA_SALU_TRIM
          const float b = (kGprIdx || FROZEN) ? bw[j] : (__builtin_amdgcn_inverse_ballot_w64(jmask[j]) ? bc : bw[j]);
#else
          const float b = (!FROZEN && j == jo && own_old) ? bc : bw[j];
#endif
          acc = __builtin_fmaf(a[j], b, acc);
          S[j] = acc;
        }

        // wavefront scan and the draw
        const float T = wave_incl_scan(acc);
        const float total = readlane_f(T, 63);
        const float thr = u * total;
        const uint64_t m = __ballot(T > thr) & last_mask;
        const int lstar = first_lane_or(m, last_lane);
        // T of lane lstar - 1 (0 for lane 0): the scan shifted one lane up
        const float E = readlane_f(dpp_mov<0x138, 0xf, true>(T), lstar);
        // every lane counts its own prefix against lane lstar's E; lstar's count is the one used
#if LDA_SALU_COUNT
        // one compare per element straight into a lane mask, and lane l*'s
        // bit added on the scalar unit (s_bitcmp1 + s_addc): 12 VALU for the
        // count at C = 8 instead of 21
        int cnt = 0;
        if constexpr (C >= 2) {
#pragma unroll
          for (int j = 0; j < C; j += 2) {
            const pkf32 es = (pkf32){E, E} + (pkf32){S[j], S[j + 1]};
            cnt = add_lane_bit(cnt, __ballot(es.x <= thr), lstar);
            cnt = add_lane_bit(cnt, __ballot(es.y <= thr), lstar);
          }
        } else {
          cnt = add_lane_bit(cnt, __ballot(E + S[0] <= thr), lstar);
        }
#else
        int cl = 0;
        if constexpr (C >= 2) {
          // E + S_j in packed pairs (each half an IEEE add)
#pragma unroll
          for (int j = 0; j < C; j += 2) {
            const pkf32 es = (pkf32){E, E} + (pkf32){S[j], S[j + 1]};
            cl += (es.x <= thr) ? 1 : 0;
            cl += (es.y <= thr) ? 1 : 0;
          }
        } else {
          cl = (E + S[0] <= thr) ? 1 : 0;
        }
        const int cnt = readlane_i(cl, lstar);
#endif
        // cnt in [0, last valid topic of lstar] or C (padded topics add 0)
        const int lim = lstar < last_lane ? C - 1 : last_j_tail;
        const int jsel = cnt < lim ? cnt : lim;
        const int kn = lstar * C + jsel;

        // the token goes back under kn with the next token's update
        kp = kn;
        inc = 1;
        // lane idx <- kn under a scalar lane mask (no per-lane compare)
        cn = __builtin_amdgcn_inverse_ballot_w64(1ull << (uint32_t)idx) ? kn : cn;
        if constexpr (!FROZEN && !LDA_CHUNK_DELTA) {
#if LDA_UPD_MASK
          // lanes 0 and 1 when the topic changed: one s_cmp + s_cselect; the
          // 32-bit cell index is valid because lda_create keeps V*Kp < 2^32
          if (__builtin_amdgcn_inverse_ballot_w64(select_mask_ne(kn, zo, lt2_mask))) {
            const int k = lane == 0 ? zo : kn;
            const int v = lane == 0 ? -1 : 1;
            atomicAdd(p.delta + ((uint32_t)w * (uint32_t)KP + (uint32_t)k), v);
            atomicAdd(&bsum[k], v);
          }
#else
          if (kn != zo && lane < 2) {
            const int k = lane == 0 ? zo : kn;
            const int v = lane == 0 ? -1 : 1;
            atomicAdd(&p.delta[(int64_t)w * KP + k], v);
            atomicAdd(&bsum[k], v);
          }
#endif
        }

    };
    // keep the pipeline full: the row of token t+P into slot s
    auto prefetch = [&](const int t, const int s) __attribute__((always_inline)) {
      const int idx = (t - cbase) & 63;
      const int wp = readlane_i(pw, idx) & kWordMask;
      load_row16<C>(rows[s], nw16 + (int64_t)wp * KP, lane);
      if (!FROZEN && !kInvM1Lds) cinv_r[s] = inv_m1[readlane_i(pz, idx)];
    };
    // The prefetch is issued for every slot, also past the range end (pw/pz
    // hold stale but valid word / topic ids there), and the loop has no exit
    // inside a group: every CFG path round the loop then issues the same P
    // row loads, and the compiler waits vmcnt(P-1) for a row instead of 0
    // (an early break becomes a flag path that skips a slot's load)
    for (int tb = 0; tb < nt; tb += P) {
#pragma unroll
      for (int s = 0; s < P; ++s) {
        if (tb + s < nt) token(tb + s, s);
        prefetch(tb + s, s);
      }
    }
    if (cbase + lane < nt) zr[cbase + lane] = cn;
    flush_delta(cw & kWordMask, cz, cn);   // lanes past the range end keep cn == cz
#pragma unroll
    for (int j = 0; j < C; ++j) nd[lane * C + j] = 0;
    wave_lds_fence();
  }

  if (!FROZEN && p.dsum) {
    __syncthreads();
    for (int i = threadIdx.x; i < KP; i += 256) {
      const int v = bsum[i];
      if (v != 0) atomicAdd(&p.dsum[i], v);
    }
  }
}

// ------------------------------------------- the half-wave dense sampler
// An opt-in variant of the dense draw for K <= 128 (lda_capi.cpp:
// LDA_DENSE_HALF=1; oracle exact_draw_half): two documents per wavefront.
// Measured on C2 (K = 128) it is slower than k_sample<2>: 8.29 vs 9.60e9
// tokens/s, VALU per token 69.7 vs 50.6 while SALU fell 45.5 -> 31.0
// (profiles/r02/half_wave/).
// K <= 128: two documents per wavefront.  Each 32-lane half runs its own
// stream of work ranges (its own chunk registers, document counts and row
// prefetches) and draws one token per step, so the per-token chain (LDS
// round trip, scan, ballot, lane select, count) is paid once for two tokens.
// Half-lane l (l = lane & 31) owns topics [l*CH, l*CH+CH), CH = 1, 2, 4 for
// K <= 32, 64, 128; the draw is exact_draw_half of the oracle:
//   S_j  = fma(a_j, b_j, S_{j-1})            (serial inside the half-lane)
//   T    = 32-lane inclusive scan: row_shr 1,2,4,8 inside 16-lane rows, then
//          row_bcast:15 into the half's second row
//   thr  = u * T_31;  l* = first half-lane <= last with T > thr (else last)
//   j*   = #{j : T_{l*-1} + S_j <= thr} clamped to the last valid topic
// The per-half scalars (token index, chunk base, document end, next topic
// to add back) are wave-uniform pairs; values the vector draw needs per
// lane (u, thr, E, the new topic) are selected by half.  A half whose queue
// ran dry idles (its draws write nothing) until the other half finishes.
constexpr uint64_t kHalf0 = 0x00000000FFFFFFFFull;

template <int CH>
__device__ __forceinline__ void load_row16_half(uint32_t (&r)[(CH + 1) / 2], const uint16_t* __restrict__ p) {
  if constexpr (CH == 4) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    r[0] = v.x;
    r[1] = v.y;
  } else if constexpr (CH == 2) {
    r[0] = *reinterpret_cast<const uint32_t*>(p);
  } else {
    r[0] = p[0];
  }
}

// 32-lane inclusive scan inside each half (exact_draw_half's order)
__device__ __forceinline__ float half_incl_scan(float x) {
  x = dpp_mov<0x111, 0xf, true>(x) + x;
  x = dpp_mov<0x112, 0xf, true>(x) + x;
  x = dpp_mov<0x114, 0xf, true>(x) + x;
  x = dpp_mov<0x118, 0xf, true>(x) + x;
  asm("s_nop 1\n\tv_add_f32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf" : "+v"(x));
  return x;
}

template <int CH, int P, bool FROZEN>
__global__ __launch_bounds__(256) void k_sample_half(SampleParams p) {
  if (p.state_dev) {                                  // a graph-launched sweep (lda_sweep)
    p.c2 = p.state_dev[0];
    p.beta = __uint_as_float(p.state_dev[1]);
  }
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  constexpr int KH = 32 * CH;                        // topics a half covers
  constexpr int KP = KH < 64 ? 64 : KH;              // row stride of nw / nw16
  constexpr int HD = (CH + 1) / 2;                   // dwords of a 16-bit row per lane
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int hl = lane & 31;
  const bool hi = lane >= 32;
  float* t_alpha = reinterpret_cast<float*>(smem);   // [KP] per block
  int32_t* bsum = smem + KP;                         // [KP] per-block nwsum delta
  float* t_invm1 = reinterpret_cast<float*>(smem + 2 * KP);  // [KP]
  // per wave and half: live doc counts nd[KH] and a = float(nd) + alpha [KH]
  int32_t* ndw = smem + 3 * KP + wid * 4 * KH;
  int32_t* nd_l = ndw + (hi ? 2 * KH : 0);           // this lane's half
  float* av_l = reinterpret_cast<float*>(nd_l + KH);

  for (int i = threadIdx.x; i < KP; i += 256) {
    t_alpha[i] = p.alpha[i];
    bsum[i] = 0;
    t_invm1[i] = FROZEN ? 0.0f : p.inv_m1[i];
  }
  for (int i = threadIdx.x; i < 16 * KH; i += 256) smem[3 * KP + i] = 0;
  __syncthreads();

  float inv_r[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) inv_r[j] = p.inv[hl * CH + j];
  const float beta = p.beta;
  const int last_lane = (p.K - 1) / CH;
  const int last_j_tail = (p.K - 1) % CH;
  const uint64_t last_mask = __ballot(hl <= last_lane);
  const uint16_t* __restrict__ nw16 = p.nw16;
  const uint8_t* __restrict__ wide_of = p.wide;
  const int32_t* __restrict__ nw = p.nw;
  constexpr int kWordMask = 0x7FFFFFFF;

  // per-half uniform state (two structs, not arrays: an array indexed by
  // half was kept in vector registers and every check became a VALU compare)
  struct Half {
    int64_t t0, doc;
    int nt, t, cbase, doc_end, ev, kp, inc;
    int active, loaded;
  };
  Half H0 = {0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 0};
  Half H1 = H0;
  // chunk registers: lane hl of half h <-> token HS(h).cbase + hl of its range
  // (words carry the int32-row flag in bit 31), the next two chunks, and the
  // word of token HS(h).cbase + hl + P for the prefetch
  int cw = 0, cz = 0, cn = 0, w1 = 0, z1 = 0, w2 = 0, z2 = 0, pw = 0;
  float cu = 0.0f;
  uint32_t rows[P][HD];
#pragma unroll
  for (int s = 0; s < P; ++s)
#pragma unroll
    for (int q = 0; q < HD; ++q) rows[s][q] = 0u;

#define HS(h) ((h) == 0 ? H0 : H1)
  // lane i of the half <- x of half-lane i + S (across the next chunk)
  auto half_shift = [&](int a, int b) -> int {
    const int src = (lane & 32) | ((hl + P) & 31);
    const int va = __shfl(a, src), vb = __shfl(b, src);
    return hl + P < 32 ? va : vb;
  };
  // the half's finished chunk: new z out, count changes into the delta
  auto flush_chunk = [&](int h) {
    if ((lane >> 5) == h) {
      const int n = HS(h).nt - HS(h).cbase;
      if (hl < n) p.z[HS(h).t0 + HS(h).cbase + hl] = cn;
      if (!FROZEN && p.delta && cn != cz) {
        const uint32_t row = (uint32_t)(cw & kWordMask) * (uint32_t)KP;
        atomicAdd(p.delta + (row + (uint32_t)cz), -1);
        atomicAdd(p.delta + (row + (uint32_t)cn), 1);
        atomicAdd(&bsum[cz], -1);
        atomicAdd(&bsum[cn], 1);
      }
    }
  };
  auto build_doc = [&](int h, int from) {
    const int32_t* zr = p.z + HS(h).t0;
    if ((lane >> 5) == h) {
      for (int i = from + hl; i < HS(h).doc_end; i += 32) atomicAdd(&nd_l[zr[i]], 1);
    }
    wave_lds_fence();
    if ((lane >> 5) == h) {
#pragma unroll
      for (int j = 0; j < CH; ++j) av_l[hl * CH + j] = (float)nd_l[hl * CH + j] + t_alpha[hl * CH + j];
    }
    wave_lds_fence();
  };
  auto clear_doc = [&](int h) {
    if ((lane >> 5) == h) {
#pragma unroll
      for (int j = 0; j < CH; ++j) nd_l[hl * CH + j] = 0;
    }
    wave_lds_fence();
  };
  // rows of tokens HS(h).t .. HS(h).t+P-1 of half h into slots s0, s0+1, ...
  auto prime = [&](int h, int s0) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int wp = readlane_i(cw, 32 * h + j) & kWordMask;   // chunk 0 holds >= P tokens' ids
      if ((lane >> 5) == h) load_row16_half<CH>(rows[(s0 + j) % P], nw16 + (int64_t)wp * KP + hl * CH);
    }
  };
  // the next work range of half h (or idle when the queue is empty)
  auto next_range = [&](int h, int s0) {
    while (true) {
      int r = 0;
      if (lane == 32 * h) r = atomicAdd(p.queue, 1);
      r = readlane_i(r, 32 * h);
      if (r >= p.num_ranges) {
        HS(h).active = 0;
        HS(h).loaded = 0;
        HS(h).ev = 0x7FFFFFFF;
        HS(h).inc = 0;
        HS(h).t = 0;                 // an idle half draws token 0 of a zero chunk
        HS(h).cbase = 0;
        HS(h).nt = 0;
        if ((lane >> 5) == h) {
          cw = 0;
          cz = 0;
          cn = 0;
        }
        return;
      }
      const int64_t d0 = p.range_doc[r], d1 = p.range_end[r];
      const int64_t s = p.doc_off[d0];
      const int n = (int)(p.doc_off[d1] - s);
      if (n <= 0) continue;
      HS(h).t0 = uniform_l(s);
      HS(h).nt = uniform_i(n);
      HS(h).t = 0;
      HS(h).cbase = 0;
      HS(h).loaded = 1;
      const int32_t* wrd = p.words + s;
      const int32_t* zr = p.z + s;
      if ((lane >> 5) == h) {
        cw = hl < n ? wrd[hl] : 0;
        cz = hl < n ? zr[hl] : 0;
        w1 = 32 + hl < n ? wrd[32 + hl] : 0;
        z1 = 32 + hl < n ? zr[32 + hl] : 0;
        w2 = 64 + hl < n ? wrd[64 + hl] : 0;
        z2 = 64 + hl < n ? zr[64 + hl] : 0;
        cw |= (int)wide_of[cw] << 31;
        w1 |= (int)wide_of[w1] << 31;
        cn = cz;
        cu = u01(draw_u32((uint64_t)(p.token_base + s + hl), p.c2, p.c3, p.k0, p.k1));
      }
      const int sh = half_shift(cw, w1);
      if ((lane >> 5) == h) pw = sh;
      int64_t dd = d0;
      while (p.doc_off[dd + 1] <= s) ++dd;
      HS(h).doc = uniform_l(dd);
      HS(h).doc_end = uniform_i((int)(p.doc_off[dd + 1] - s));
      build_doc(h, 0);
      HS(h).inc = 0;
      HS(h).ev = uniform_i(min(32, HS(h).doc_end));
      prime(h, s0);
      return;
    }
  };
  auto event = [&](int h, int s0) {
    if (HS(h).t == HS(h).nt) {
      // the range is done (or none was loaded yet)
      if (HS(h).loaded) {
        flush_chunk(h);
        clear_doc(h);
      }
      next_range(h, s0);
      return;
    }
    if (HS(h).t - HS(h).cbase == 32) {
      flush_chunk(h);
      HS(h).cbase = uniform_i(HS(h).cbase + 32);
      const int n = HS(h).nt;
      const int32_t* wrd = p.words + HS(h).t0;
      const int32_t* zr = p.z + HS(h).t0;
      if ((lane >> 5) == h) {
        cw = w1;
        cz = z1;
        w1 = w2;
        z1 = z2;
        w1 |= (int)wide_of[w1] << 31;
        cn = cz;
        cu = u01(draw_u32((uint64_t)(p.token_base + HS(h).t0 + HS(h).cbase + hl), p.c2, p.c3, p.k0, p.k1));
        if (HS(h).cbase + 64 + hl < n) {
          w2 = wrd[HS(h).cbase + 64 + hl];
          z2 = zr[HS(h).cbase + 64 + hl];
        }
      }
      const int sh = half_shift(cw, w1);
      if ((lane >> 5) == h) pw = sh;
    }
    if (HS(h).t == HS(h).doc_end) {
      HS(h).inc = 0;                 // the pending add-back belonged to the last document
      clear_doc(h);
      int64_t dd = HS(h).doc + 1;
      while (p.doc_off[dd + 1] - HS(h).t0 <= HS(h).t) ++dd;
      HS(h).doc = uniform_l(dd);
      HS(h).doc_end = uniform_i((int)(p.doc_off[dd + 1] - HS(h).t0));
      build_doc(h, HS(h).t);
    }
    HS(h).ev = uniform_i(min(HS(h).cbase + 32, HS(h).doc_end));
  };

  while (true) {
#pragma unroll
    for (int s = 0; s < P; ++s) {
#pragma unroll
      for (int h = 0; h < 2; ++h)
        if (HS(h).t == HS(h).ev) event(h, s);
      if (!H0.active && !H1.active) goto done;

      // ---- one token of each half
      const int idx0 = H0.t - H0.cbase, idx1 = H1.t - H1.cbase;
      const int wf0 = readlane_i(cw, idx0), wf1 = readlane_i(cw, 32 + idx1);
      const int zo0 = readlane_i(cz, idx0), zo1 = readlane_i(cz, 32 + idx1);
      const float u0 = readlane_f(cu, idx0), u1 = readlane_f(cu, 32 + idx1);
      const int zo_l = hi ? zo1 : zo0;

      // lanes 0 / 32: add the previous token of the half back under kp
      // (deferred from its draw), then remove this one
      if (hl == 0 && (hi ? H1.active : H0.active)) {
        const int k = hi ? H1.kp : H0.kp;
        const int ndk = nd_l[k] + (hi ? H1.inc : H0.inc);
        nd_l[k] = ndk;
        av_l[k] = (float)ndk + t_alpha[k];
        const int ndz = nd_l[zo_l] - 1;
        nd_l[zo_l] = ndz;
        av_l[zo_l] = (float)ndz + t_alpha[zo_l];
      }
      wave_lds_fence();
      float a[CH];
      load_lds_f<CH>(a, av_l + hl * CH);
      const float cinv = FROZEN ? 0.0f : t_invm1[zo_l];

      // counts of the row (16-bit, or the int32 row for a word with a count
      // > 65535: rare, uniform per half, drained in its branch)
      int32_t cfull[CH];
      const bool wide0 = wf0 < 0, wide1 = wf1 < 0;
      if (wide0 || wide1) {
        const bool mine = hi ? wide1 : wide0;
        const int wl = (hi ? wf1 : wf0) & kWordMask;
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int c16 = (j & 1) ? (int)(rows[s][j >> 1] >> 16) : (int)(rows[s][j >> 1] & 0xFFFFu);
          cfull[j] = mine ? nw[(int64_t)wl * KP + hl * CH + j] : (CH == 1 ? (int)rows[s][0] : c16);
        }
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
      } else {
        if constexpr (CH == 1) {
          cfull[0] = (int32_t)rows[s][0];
        } else {
#pragma unroll
          for (int j = 0; j < CH; ++j)
            cfull[j] = (j & 1) ? (int32_t)(rows[s][j >> 1] >> 16) : (int32_t)(rows[s][j >> 1] & 0xFFFFu);
        }
      }
      // own-token correction: topic zo of each half, one vector compare per
      // element against the lane's half's z_old (the scalar unit is the
      // scarce one here)
      bool own[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) own[j] = !FROZEN && (hl * CH + j == zo_l);
      int32_t c_old = cfull[0];
#pragma unroll
      for (int j = 1; j < CH; ++j) c_old = own[j] ? cfull[j] : c_old;
      const float bc = FROZEN ? 0.0f : ((float)(c_old - 1) + beta) * cinv;
      float S[CH];
      float acc = 0.0f;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const float bw = ((float)cfull[j] + beta) * inv_r[j];
        const float b = own[j] ? bc : bw;
        acc = __builtin_fmaf(a[j], b, acc);
        S[j] = acc;
      }

      // the half scans and the two draws
      const float T = half_incl_scan(acc);
      const float thr0 = u0 * readlane_f(T, 31), thr1 = u1 * readlane_f(T, 63);
      const float thr = hi ? thr1 : thr0;
      const uint64_t m = __ballot(T > thr) & last_mask;
      const int ls0 = first_lane_or(m & kHalf0, last_lane);
      const int ls1 = first_lane_or(m >> 32, last_lane);
      const float Tsh = dpp_mov<0x138, 0xf, true>(T);      // wave_shr:1
      const float E0 = ls0 > 0 ? readlane_f(Tsh, ls0) : 0.0f;
      const float E1 = ls1 > 0 ? readlane_f(Tsh, 32 + ls1) : 0.0f;
      const float E = hi ? E1 : E0;
      // each lane counts its own prefix; lane l* of each half is read
      int cl = 0;
#pragma unroll
      for (int j = 0; j < CH; ++j) cl += (E + S[j] <= thr) ? 1 : 0;
      const int cnt0 = readlane_i(cl, ls0), cnt1 = readlane_i(cl, 32 + ls1);
      const int lim0 = ls0 < last_lane ? CH - 1 : last_j_tail;
      const int lim1 = ls1 < last_lane ? CH - 1 : last_j_tail;
      const int kn0 = ls0 * CH + (cnt0 < lim0 ? cnt0 : lim0);
      const int kn1 = ls1 * CH + (cnt1 < lim1 ? cnt1 : lim1);

      // the token goes back under kn with the half's next token; lane idx of
      // each active half takes its new topic
      const uint64_t upd = (H0.active ? (1ull << (uint32_t)idx0) : 0ull) |
                           (H1.active ? (1ull << (uint32_t)(32 + idx1)) : 0ull);
      cn = __builtin_amdgcn_inverse_ballot_w64(upd) ? (hi ? kn1 : kn0) : cn;
      H0.kp = uniform_i(kn0);
      H1.kp = uniform_i(kn1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        HS(h).inc = HS(h).active ? 1 : 0;
        HS(h).t = uniform_i(HS(h).t + (HS(h).active ? 1 : 0));
      }

      // keep the pipeline full: the rows of each half's token t + P - 1 + 1
      {
        const int pi0 = (H0.t - 1 - H0.cbase) & 31, pi1 = (H1.t - 1 - H1.cbase) & 31;
        const int wp0 = readlane_i(pw, pi0) & kWordMask, wp1 = readlane_i(pw, 32 + pi1) & kWordMask;
        const int wp = hi ? wp1 : wp0;
        load_row16_half<CH>(rows[s], nw16 + (int64_t)wp * KP + hl * CH);
      }
    }
  }
done:
#undef HS
  if (!FROZEN && p.dsum) {
    __syncthreads();
    for (int i = threadIdx.x; i < KP; i += 256) {
      const int v = bsum[i];
      if (v != 0) atomicAdd(&p.dsum[i], v);
    }
  }
}

// ------------------------------------------ the quarter-wave dense sampler
// K <= 128: four documents per wavefront, one per 16-lane DPP row.  Each row
// (quarter) runs its own stream of work ranges; every per-document quantity
// is a per-lane vector that is uniform inside the row (token index, chunk
// base, document end, next topic to add back), so one step draws one token of
// each quarter with row-local DPP (scan, broadcast) and ds_bpermute instead of
// the full-wave kernel's scalar unit.  Row-lane l owns topics [l*CH, l*CH+CH),
// CH = 1, 2, 4, 8 for K <= 16, 32, 64, 128 (oracle exact_draw_quarter):
//   S_j = fma(a_j, b_j, S_{j-1});  T = inclusive row scan (row_shr 1,2,4,8)
//   thr = u * T_15;  l* = first row-lane <= last with T > thr (else last)
//   j*  = #{j : T_{l*-1} + S_j <= thr} clamped to the last valid topic
template <int CH>
__device__ __forceinline__ void load_row16_q(uint32_t (&r)[(CH + 1) / 2], const uint16_t* __restrict__ p) {
  if constexpr (CH == 8) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    r[0] = v.x;
    r[1] = v.y;
    r[2] = v.z;
    r[3] = v.w;
  } else if constexpr (CH == 4) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    r[0] = v.x;
    r[1] = v.y;
  } else if constexpr (CH == 2) {
    r[0] = *reinterpret_cast<const uint32_t*>(p);
  } else {
    r[0] = p[0];
  }
}
template <int CH>
__device__ __forceinline__ uint32_t qrow_first16(const uint32_t (&r)[(CH + 1) / 2]) {
  return r[0] & 0xFFFFu;
}
__device__ __forceinline__ int row_bcast15_i(int v) { return __builtin_amdgcn_update_dpp(0, v, 0x15F, 0xF, 0xF, false); }
__device__ __forceinline__ float row_bcast15_f(float v) {
  return __builtin_bit_cast(float, row_bcast15_i(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float row_scan16_q(float x) {
  x = dpp_mov<0x111, 0xf, true>(x) + x;
  x = dpp_mov<0x112, 0xf, true>(x) + x;
  x = dpp_mov<0x114, 0xf, true>(x) + x;
  x = dpp_mov<0x118, 0xf, true>(x) + x;
  return x;
}
__device__ __forceinline__ int row_scan16_i(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  return x;
}
// lane (row base + i) of v, i per lane (ds_bpermute)
__device__ __forceinline__ int row_get_i(int v, int rowbase, int i) {
  return __builtin_amdgcn_ds_bpermute((rowbase + i) << 2, v);
}
__device__ __forceinline__ float row_get_f(float v, int rowbase, int i) {
  return __builtin_bit_cast(float, row_get_i(__builtin_bit_cast(int, v), rowbase, i));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int CH, int P, bool FROZEN>
// 5 waves per SIMD for the training kernel (96 VGPRs + 24 B/lane of spill
// at CH = 8): +7% on C2 after burn-in, equal near
// init, over the unconstrained 108 VGPRs / 4 waves; 6 waves spill 76 B and
// lose 25% (profiles/r02/quarter/ab).  The frozen kernel fits 5 unforced.
#ifndef QUARTER_WPE
#define QUARTER_WPE 5
#endif
// 1: the word factors and the prefix-count sums two topics per packed fp32
// instruction (round 6 A/B)
#ifndef QUARTER_PK
#define QUARTER_PK 0
#endif
#define QUARTER_ATTR __attribute__((amdgpu_waves_per_eu(FROZEN ? 4 : QUARTER_WPE)))
__global__ __launch_bounds__(256) QUARTER_ATTR void k_sample_quarter(SampleParams p) {
  if (p.state_dev) {                                  // a graph-launched sweep (lda_sweep)
    p.c2 = p.state_dev[0];
    p.beta = __uint_as_float(p.state_dev[1]);
  }
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  constexpr int KQ = 16 * CH;                        // topics a quarter covers
  constexpr int KP = KQ < 64 ? 64 : KQ;              // row stride of nw / nw16
  constexpr int HD = (CH + 1) / 2;                   // dwords of a 16-bit row per lane
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int ql = lane & 15;
  const int rb = lane & 48;                          // the row's first lane
  float* t_alpha = reinterpret_cast<float*>(smem);   // [KP] per block
  int32_t* bsum = smem + KP;                         // [KP] per-block nwsum delta
  float* t_invm1 = reinterpret_cast<float*>(smem + 2 * KP);
  // per wave and quarter: live doc counts nd[KQ] and a = float(nd) + alpha [KQ]
  int32_t* nd_l = smem + 3 * KP + wid * 8 * KQ + (lane >> 4) * 2 * KQ;
  float* av_l = reinterpret_cast<float*>(nd_l + KQ);

  for (int i = threadIdx.x; i < KP; i += 256) {
    t_alpha[i] = p.alpha[i];
    bsum[i] = 0;
    t_invm1[i] = FROZEN ? 0.0f : p.inv_m1[i];
  }
  for (int i = threadIdx.x; i < 32 * KQ; i += 256) smem[3 * KP + i] = 0;
  __syncthreads();

  float inv_r[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) inv_r[j] = p.inv[ql * CH + j];
  const float beta = p.beta;
  const int last_lane = (p.K - 1) / CH;
  const int last_j_tail = (p.K - 1) % CH;
  const uint16_t* __restrict__ nw16 = p.nw16;
  const int32_t* __restrict__ nw = p.nw;

  // per-quarter state, uniform inside each row
  int64_t t0 = 0, doc = 0;
  int nt = 0, t = 0, cbase = 0, doc_end = 0, ev = 0, kp = 0, inc = 0;
  int active = 1, loaded = 0;
  bool first_range = true;                           // per row (lane-varying)
  // chunk registers: row-lane i <-> token cbase + i of the quarter's range
  int cw = 0, cz = 0, cn = 0, w1 = 0, z1 = 0, w2 = 0, z2 = 0, pw = 0;
  uint32_t cpos = 0;                                 // zw position of the chunk's token (recount sweeps)
  float cu = 0.0f;
  uint32_t rows[P][HD];
#pragma unroll
  for (int s = 0; s < P; ++s)
#pragma unroll
    for (int q = 0; q < HD; ++q) rows[s][q] = 0u;

  auto shift_words = [&]() {        // word of token cbase + i + P (across chunks)
    const int src = ql + P;
    const int va = row_get_i(cw, rb, src & 15), vb = row_get_i(w1, rb, src & 15);
    pw = src < 16 ? va : vb;
  };

  while (true) {
#pragma unroll
    for (int s = 0; s < P; ++s) {
      // ---- events of the quarters that reached one (lanes of those rows)
      if (__ballot(active && t == ev) != 0) {
        if (active && t == ev) {
          if (t == nt) {
            // the range is done (or none loaded yet): publish, clear, next range
            if (loaded) {
              if (ql < nt - cbase) p.z[t0 + cbase + ql] = cn;
              if (!FROZEN && p.zw && cn != cz && ql < nt - cbase) p.zw[cpos] = cn;
              if (!FROZEN && p.delta && cn != cz) {
                const uint32_t row = (uint32_t)cw * (uint32_t)KP;
                atomicAdd(p.delta + (row + (uint32_t)cz), -1);
                atomicAdd(p.delta + (row + (uint32_t)cn), 1);
                atomicAdd(&bsum[cz], -1);
                atomicAdd(&bsum[cn], 1);
              }
#pragma unroll
              for (int j = 0; j < CH; ++j) nd_l[ql * CH + j] = 0;
            }
            loaded = 0;
            while (true) {
              int r = 0;
              if ((!LDA_STATIC_FIRST || !first_range) && ql == 0) r = atomicAdd(p.queue, 1);
              r = first_or_queued(first_range, ((int)blockIdx.x * 4 + wid) * 4 + (lane >> 4),
                                  (int)gridDim.x * 16, row_get_i(r, rb, 0));
              first_range = false;
              if (r >= p.num_ranges) {
                active = 0;
                ev = -1;
                t = 0;
                cbase = 0;
                nt = 0;
                inc = 0;
                kp = 0;
                cw = 0;
                cz = 0;
                cn = 0;
                pw = 0;
                break;
              }
              const int64_t d0 = p.range_doc[r], d1 = p.range_end[r];
              const int64_t s0 = p.doc_off[d0];
              const int n = (int)(p.doc_off[d1] - s0);
              if (n <= 0) continue;
              t0 = s0;
              nt = n;
              t = 0;
              cbase = 0;
              loaded = 1;
              const int32_t* wrd = p.words + s0;
              const int32_t* zr = p.z + s0;
              cw = ql < n ? wrd[ql] : 0;
              cz = ql < n ? zr[ql] : 0;
              w1 = 16 + ql < n ? wrd[16 + ql] : 0;
              z1 = 16 + ql < n ? zr[16 + ql] : 0;
              w2 = 32 + ql < n ? wrd[32 + ql] : 0;
              z2 = 32 + ql < n ? zr[32 + ql] : 0;
              cn = cz;
              if (!FROZEN && p.zw && ql < n) cpos = p.zpos[s0 + ql];   // used at the chunk's publish
              cu = u01(draw_u32((uint64_t)(p.token_base + s0 + ql), p.c2, p.c3, p.k0, p.k1));
              int64_t dd = d0;
              while (p.doc_off[dd + 1] <= s0) ++dd;
              doc = dd;
              doc_end = (int)(p.doc_off[dd + 1] - s0);
              break;
            }
            if (active) {
              shift_words();
              const int32_t* zr = p.z + t0;
              for (int i = ql; i < doc_end; i += 16) atomicAdd(&nd_l[zr[i]], 1);
              wave_lds_fence();
#pragma unroll
              for (int j = 0; j < CH; ++j) av_l[ql * CH + j] = (float)nd_l[ql * CH + j] + t_alpha[ql * CH + j];
              inc = 0;
              ev = min(16, doc_end);
              // rows of the range's first P tokens into slots s, s+1, ...
#pragma unroll
              for (int j = 0; j < P; ++j) {
                const int wp = row_get_i(cw, rb, j);
                load_row16_q<CH>(rows[(s + j) % P], nw16 + (int64_t)wp * KP + ql * CH);
              }
            }
          } else {
            if (t - cbase == 16) {
              // chunk switch: publish the finished chunk, shift
              p.z[t0 + cbase + ql] = cn;
              if (!FROZEN && p.zw && cn != cz) p.zw[cpos] = cn;
              if (!FROZEN && p.delta && cn != cz) {
                const uint32_t row = (uint32_t)cw * (uint32_t)KP;
                atomicAdd(p.delta + (row + (uint32_t)cz), -1);
                atomicAdd(p.delta + (row + (uint32_t)cn), 1);
                atomicAdd(&bsum[cz], -1);
                atomicAdd(&bsum[cn], 1);
              }
              cbase += 16;
              cw = w1;
              cz = z1;
              w1 = w2;
              z1 = z2;
              cn = cz;
              if (!FROZEN && p.zw && cbase + ql < nt) cpos = p.zpos[t0 + cbase + ql];
              cu = u01(draw_u32((uint64_t)(p.token_base + t0 + cbase + ql), p.c2, p.c3, p.k0, p.k1));
              if (cbase + 32 + ql < nt) {
                w2 = p.words[t0 + cbase + 32 + ql];
                z2 = p.z[t0 + cbase + 32 + ql];
              }
              shift_words();
            }
            if (t == doc_end) {
              inc = 0;               // the pending add-back belonged to the last document
#pragma unroll
              for (int j = 0; j < CH; ++j) nd_l[ql * CH + j] = 0;
              wave_lds_fence();
              int64_t dd = doc + 1;
              while (p.doc_off[dd + 1] - t0 <= t) ++dd;
              doc = dd;
              doc_end = (int)(p.doc_off[dd + 1] - t0);
              const int32_t* zr = p.z + t0;
              for (int i = t + ql; i < doc_end; i += 16) atomicAdd(&nd_l[zr[i]], 1);
              wave_lds_fence();
#pragma unroll
              for (int j = 0; j < CH; ++j) av_l[ql * CH + j] = (float)nd_l[ql * CH + j] + t_alpha[ql * CH + j];
            }
            ev = min(cbase + 16, doc_end);
          }
        }
        wave_lds_fence();
      }
      if (__ballot(active) == 0) goto done;

      // ---- one token of every quarter
      const int idx = t - cbase;
      const int wf = row_get_i(cw, rb, idx);
      const int zo = row_get_i(cz, rb, idx);
      const float u = row_get_f(cu, rb, idx);
      // the document factors a_k as running fp32 values (oracle
      // exact_draw_quarter): +1 for the previous token's new topic, -1 for this
      // token's old one, as LDS float atomics (in order, nothing to wait for)
      if (ql == 0 && active) {
        atomicAdd(&av_l[kp], (float)inc);
        atomicAdd(&av_l[zo], -1.0f);
      }
      wave_lds_fence();
      float a[CH];
      load_lds_f<CH>(a, av_l + ql * CH);
      const float cinv = FROZEN ? 0.0f : t_invm1[zo];

      int32_t cfull[CH];
      // the int32 row where this lane's first 16-bit count is 0xFFFF: a wide
      // word's row is all 0xFFFF (k_apply_packed); a true count of 65535
      // takes the int32 row too, which holds the same value
      const bool wide = (qrow_first16<CH>(rows[s])) == 0xFFFFu;
      if (__ballot(wide) != 0) {
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const int c16 = CH == 1 ? (int)rows[s][0] : ((j & 1) ? (int)(rows[s][j >> 1] >> 16) : (int)(rows[s][j >> 1] & 0xFFFFu));
          cfull[j] = wide ? nw[(int64_t)wf * KP + ql * CH + j] : c16;
        }
        __builtin_amdgcn_s_waitcnt(kVmcnt0);
      } else {
        if constexpr (CH == 1) {
          cfull[0] = (int32_t)rows[s][0];
        } else {
#pragma unroll
          for (int j = 0; j < CH; ++j)
            cfull[j] = (j & 1) ? (int32_t)(rows[s][j >> 1] >> 16) : (int32_t)(rows[s][j >> 1] & 0xFFFFu);
        }
      }
      bool own[CH];
#pragma unroll
      for (int j = 0; j < CH; ++j) own[j] = !FROZEN && (ql * CH + j == zo);
      int32_t c_old = cfull[0];
#pragma unroll
      for (int j = 1; j < CH; ++j) c_old = own[j] ? cfull[j] : c_old;
      const float bc = FROZEN ? 0.0f : ((float)(c_old - 1) + beta) * cinv;
      float S[CH];
      float acc = 0.0f;
#if QUARTER_PK
      // the word factors two topics per instruction (v_pk_add_f32 /
      // v_pk_mul_f32: the same IEEE operations, element for element)
      float bw[CH];
#pragma unroll
      for (int j = 0; j < CH; j += 2) {
        if (j + 1 < CH) {
          const f32x2 cf = {(float)cfull[j], (float)cfull[j + 1]};
          const f32x2 iv = {inv_r[j], inv_r[j + 1]};
          const f32x2 bb = {beta, beta};
          const f32x2 r = (cf + bb) * iv;
          bw[j] = r.x;
          bw[j + 1] = r.y;
        } else {
          bw[j] = ((float)cfull[j] + beta) * inv_r[j];
        }
      }
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        acc = __builtin_fmaf(a[j], own[j] ? bc : bw[j], acc);
        S[j] = acc;
      }
#else
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const float bw = ((float)cfull[j] + beta) * inv_r[j];
        const float b = own[j] ? bc : bw;
        acc = __builtin_fmaf(a[j], b, acc);
        S[j] = acc;
      }
#endif
      const float T = row_scan16_q(acc);
      const float thr = u * row_bcast15_f(T);
      // l* = #{row-lanes with T <= thr} (T is monotone), clamped to the last:
      // the row's 16 bits of one ballot, counted per lane
      const uint64_t le = __ballot(T <= thr);
      const int cle = __builtin_popcount((uint32_t)(le >> rb) & 0xFFFFu);
      const int ls = min(cle, last_lane);
      // every lane's count against its left neighbour's T (0 on row-lane 0):
      // lane l*'s is the draw's (E = T_{l*-1}), fetched once
      const float E = dpp_mov<0x111, 0xf, true>(T);
      int cl = 0;
#if QUARTER_PK
      {
        const f32x2 ee = {E, E};
#pragma unroll
        for (int j = 0; j < CH; j += 2) {
          if (j + 1 < CH) {
            const f32x2 sj = {S[j], S[j + 1]};
            const f32x2 es = ee + sj;
            cl += (es.x <= thr) ? 1 : 0;
            cl += (es.y <= thr) ? 1 : 0;
          } else {
            cl += (E + S[j] <= thr) ? 1 : 0;
          }
        }
      }
#else
#pragma unroll
      for (int j = 0; j < CH; ++j) cl += (E + S[j] <= thr) ? 1 : 0;
#endif
      const int cnt = row_get_i(cl, rb, ls);
      const int lim = ls < last_lane ? CH - 1 : last_j_tail;
      const int kn = ls * CH + (cnt < lim ? cnt : lim);

      cn = (active && ql == idx) ? kn : cn;
      kp = kn;
      inc = active;
      t += active;

      // keep the pipeline full: the row of each quarter's token t + P - 1 + 1
      {
        const int wp = row_get_i(pw, rb, (t - 1 - cbase) & 15);
        load_row16_q<CH>(rows[s], nw16 + (int64_t)wp * KP + ql * CH);
      }
    }
  }
done:
  if (!FROZEN && p.dsum) {
    __syncthreads();
    for (int i = threadIdx.x; i < KP; i += 256) {
      const int v = bsum[i];
      if (v != 0) atomicAdd(&p.dsum[i], v);
    }
  }
}

// 16-bit copy of nw (+ per-word "wide" flag when a count exceeds 65535).
template <int C>
__global__ __launch_bounds__(256) void k_build_packed(const int32_t* __restrict__ nw, int64_t V,
                                                      uint16_t* __restrict__ nw16,
                                                      uint8_t* __restrict__ wide) {
  constexpr int KP = C * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * 4 + wid; w < V; w += (int64_t)gridDim.x * 4) {
    int32_t c[C];
    load_row<C>(c, nw + w * KP + lane * C);
    bool big = false;
#pragma unroll
    for (int j = 0; j < C; ++j) big |= (uint32_t)c[j] > 0xFFFFu;
    // a wide word's whole 16-bit row is 0xFFFF: the quarter kernel reads its
    // "take the int32 row" flag from the row itself (k_sample_quarter)
    const uint64_t any = __ballot(big);
#pragma unroll
    for (int j = 0; j < C; ++j)
      nw16[w * KP + lane * C + j] = any ? (uint16_t)0xFFFFu : (uint16_t)c[j];
    if (lane == 0) wide[w] = any ? 1 : 0;
  }
}

// ------------------------------------------------------ the sparse sampler
// Same semantics and Philox keying as k_sample; the categorical weights are
// split SparseLDA-style so that a token reads only the NONZERO entries of its
// word row (packed (count << 12) | topic, built per sweep by k_build_sparse):
//   coef_k = (float(nd_k) + alpha_k) * (k == z_old ? inv_m1_k : inv_k)
//   B_e    = coef[t_e] * float(c_e - [t_e == z_old])   (word part, sparse)
//   A_k    = coef_k * beta                               (doc part, dense)
// Exact fp32 order (oracle/lda_oracle.c:exact_draw_sparse): lane l holds
// entries e = l + 64r, serial add over r, DPP scan; lane l owns topics
// [l*C, l*C+C) for A, serial fma chain, DPP scan; thr = u * (sumB + sumA),
// B searched first.  coef and nd live in LDS per wave; the per-lane A
// partial is a register recomputed only for the lanes whose topics changed.
template <int C>
__device__ __forceinline__ float coef_partial(const float* __restrict__ coef_lane, float beta) {
  float a = 0.0f;
#pragma unroll
  for (int q = 0; q < C; q += 4) {
    if constexpr (C >= 4) {
      const float4 v = *reinterpret_cast<const float4*>(coef_lane + q);
      a = __builtin_fmaf(v.x, beta, a);
      a = __builtin_fmaf(v.y, beta, a);
      a = __builtin_fmaf(v.z, beta, a);
      a = __builtin_fmaf(v.w, beta, a);
    } else {
#pragma unroll
      for (int j = 0; j < C; ++j) a = __builtin_fmaf(coef_lane[j], beta, a);
    }
  }
  return a;
}

template <int C, int P, int R0, bool FROZEN>
__global__ __launch_bounds__(256) void k_sample_sparse(SampleParams p) {
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  constexpr int KP = C * 64;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float* t_alpha = reinterpret_cast<float*>(smem);  // per-block topic tables
  float* t_inv = t_alpha + KP;
  float* t_invm1 = t_inv + KP;
  int32_t* bsum = smem + 3 * KP;                    // per-block nwsum delta
  int32_t* nd = smem + 4 * KP + wid * 2 * KP;       // per-wave live doc counts
  float* coef = reinterpret_cast<float*>(nd + KP);  // per-wave coefficients

  for (int i = threadIdx.x; i < KP; i += 256) {
    t_alpha[i] = p.alpha[i];
    t_inv[i] = p.inv[i];
    t_invm1[i] = FROZEN ? 0.0f : p.inv_m1[i];
    bsum[i] = 0;
  }
  for (int i = threadIdx.x; i < 8 * KP; i += 256) smem[4 * KP + i] = 0;
  __syncthreads();

  const float beta = p.beta;
  const int last_lane = (p.K - 1) / C;
  const int last_j = (lane < last_lane) ? C - 1 : (p.K - 1) % C;
  const int32_t* __restrict__ nw = p.nw;
  const uint32_t* __restrict__ ent = p.ent;
  const int64_t* __restrict__ row_off = p.row_off;
  const int32_t* __restrict__ row_nnz = p.row_nnz;

  bool first_range = true;
  while (true) {
    int r = 0;
    if ((!LDA_STATIC_FIRST || !first_range) && lane == 0) r = atomicAdd(p.queue, 1);
    r = uniform_i(first_or_queued(first_range, (int)blockIdx.x * 4 + wid, (int)gridDim.x * 4, uniform_i(__shfl(r, 0))));
    first_range = false;
    if (r >= p.num_ranges) break;
    const int64_t d0 = p.range_doc[r], d1 = p.range_end[r];
    const int64_t t0 = p.doc_off[d0], t1 = p.doc_off[d1];
    if (t1 <= t0) continue;

    // --- chunk registers: chunk c (cw, cz, cu, cn, row meta), chunk c+1
    // (words, z, row meta), chunk c+2 (words, z).  Row meta of chunk c+1 is
    // gathered one chunk ahead, so entry prefetches never wait on it.
    int64_t cbase = t0;
    int cw = 0, cz = 0, w1 = 0, z1 = 0, w2 = 0, z2 = 0;
    if (t0 + lane < t1) {
      cw = p.words[t0 + lane];
      cz = p.z[t0 + lane];
    }
    if (t0 + 64 + lane < t1) {
      w1 = p.words[t0 + 64 + lane];
      z1 = p.z[t0 + 64 + lane];
    }
    if (t0 + 128 + lane < t1) {
      w2 = p.words[t0 + 128 + lane];
      z2 = p.z[t0 + 128 + lane];
    }
    int cmn = row_nnz[cw], m1n = row_nnz[w1];
    int64_t cmo = row_off[cw], m1o = row_off[w1];
    int cn = cz;
    float cu = u01(draw_u32((uint64_t)(p.token_base + t0 + lane), p.c2, p.c3, p.k0, p.k1));

    // --- first document of the range
    int64_t doc = d0;
    while (p.doc_off[doc + 1] <= t0) ++doc;
    int64_t doc_end = p.doc_off[doc + 1];
    float TA;
    {
      for (int64_t i = t0 + lane; i < doc_end; i += 64) atomicAdd(&nd[p.z[i]], 1);
      wave_lds_fence();
      float a = 0.0f;
#pragma unroll
      for (int j = 0; j < C; ++j) {
        const int k = lane * C + j;
        const float cf = ((float)nd[k] + t_alpha[k]) * t_inv[k];
        coef[k] = cf;
        a = __builtin_fmaf(cf, beta, a);
      }
      TA = a;
      wave_lds_fence();
    }

    // --- prime the entry pipeline: first R0 rounds of the next P tokens
    uint32_t ring[P][R0];
#pragma unroll
    for (int s = 0; s < P; ++s) {
      const int64_t tp = t0 + s;
      const int n = readlane_i(cmn, s) & 0x7FFFFFFF;
      const int64_t o = ((int64_t)readlane_i((int)(cmo >> 32), s) << 32) |
                        (uint32_t)readlane_i((int)cmo, s);
#pragma unroll
      for (int q = 0; q < R0; ++q)
        ring[s][q] = (tp < t1 && q * 64 + lane < n) ? ent[o + q * 64 + lane] : 0u;
    }

    for (int64_t tb = t0; tb < t1; tb += P) {
#pragma unroll
      for (int s = 0; s < P; ++s) {
        const int64_t t = tb + s;
        if (t >= t1) break;
        int idx = (int)(t - cbase);
        if (idx == 64) {
          p.z[cbase + lane] = cn;
          cbase += 64;
          idx = 0;
          cw = w1;
          cz = z1;
          cmn = m1n;
          cmo = m1o;
          w1 = w2;
          z1 = z2;
          m1n = row_nnz[w1];
          m1o = row_off[w1];
          cn = cz;
          cu = u01(draw_u32((uint64_t)(p.token_base + cbase + lane), p.c2, p.c3, p.k0, p.k1));
          if (cbase + 128 + lane < t1) {
            w2 = p.words[cbase + 128 + lane];
            z2 = p.z[cbase + 128 + lane];
          }
        }
        if (t == doc_end) {
#pragma unroll
          for (int j = 0; j < C; ++j) nd[lane * C + j] = 0;
          wave_lds_fence();
          ++doc;
          while (p.doc_off[doc + 1] <= t) ++doc;
          doc_end = p.doc_off[doc + 1];
          for (int64_t i = t + lane; i < doc_end; i += 64) atomicAdd(&nd[p.z[i]], 1);
          wave_lds_fence();
          float a = 0.0f;
#pragma unroll
          for (int j = 0; j < C; ++j) {
            const int k = lane * C + j;
            const float cf = ((float)nd[k] + t_alpha[k]) * t_inv[k];
            coef[k] = cf;
            a = __builtin_fmaf(cf, beta, a);
          }
          TA = a;
          wave_lds_fence();
        }

        const int w = readlane_i(cw, idx);
        const int zo = readlane_i(cz, idx);
        const float u = readlane_f(cu, idx);
        const int n_raw = readlane_i(cmn, idx);
        const bool row_sat = n_raw < 0;           // the row holds a saturated count
        const int n = n_raw & 0x7FFFFFFF;
        const int64_t off = ((int64_t)readlane_i((int)(cmo >> 32), idx) << 32) |
                            (uint32_t)readlane_i((int)cmo, idx);
        const int lo = zo / C;

        // remove the token from its document (and, unless frozen, from the
        // snapshot's row/total through inv_m1 and c - 1 below)
        {
          const int ndz = nd[zo] - 1;
          const float cf = ((float)ndz + t_alpha[zo]) * (FROZEN ? t_inv[zo] : t_invm1[zo]);
          if (lane == 0) {
            nd[zo] = ndz;
            coef[zo] = cf;
          }
          wave_lds_fence();
          if (lane == lo) TA = coef_partial<C>(coef + lane * C, beta);
        }

        // word part over the nonzero entries of row w
        uint32_t e[C];
        float SB[C];
#pragma unroll
        for (int q = 0; q < C; ++q) {
          if (q < R0)
            e[q] = ring[s][q];
          else
            e[q] = (q * 64 < n && q * 64 + lane < n) ? ent[off + q * 64 + lane] : 0u;
        }
        float accB = 0.0f;
        int tsel_r[C];
#pragma unroll
        for (int q = 0; q < C; ++q) {
          SB[q] = accB;
          tsel_r[q] = 0;
          if (q * 64 < n) {
            const bool valid = q * 64 + lane < n;
            const int tq = (int)(e[q] & ENT_TOPIC_MASK);
            int cq = (int)(e[q] >> ENT_TOPIC_BITS);
            if (row_sat && valid && (uint32_t)cq == ENT_COUNT_SAT) cq = nw[(int64_t)w * KP + tq];
            if (!FROZEN) cq -= (tq == zo) ? 1 : 0;
            const float b = valid ? coef[tq] * (float)cq : 0.0f;
            accB = accB + b;
            SB[q] = accB;
            tsel_r[q] = tq;
          }
        }
        const float TB = wave_incl_scan(accB);
        const float TAs = wave_incl_scan(TA);
        const float sumB = readlane_f(TB, 63);
        const float sumA = readlane_f(TAs, 63);
        const float thr = u * (sumB + sumA);
        int kn;
        if (thr < sumB) {
          const int nl = n < 64 ? n : 64;
          const uint64_t m = __ballot((TB > thr) && (lane < nl));
          const int lstar = m ? (int)__builtin_ctzll(m) : nl - 1;
          const float E = lstar > 0 ? readlane_f(TB, lstar - 1) : 0.0f;
          const int nr = lane < n ? (n - lane + 63) / 64 : 0;
          int cnt = 0;
#pragma unroll
          for (int q = 0; q < C; ++q)
            if (q * 64 < n) cnt += (q < nr && E + SB[q] <= thr) ? 1 : 0;
          const int rsel = cnt < nr ? cnt : nr - 1;
          int tsel = 0;
#pragma unroll
          for (int q = 0; q < C; ++q) tsel = (q == rsel) ? tsel_r[q] : tsel;
          kn = readlane_i(tsel, lstar);
        } else {
          const float thr2 = thr - sumB;
          const uint64_t m = __ballot((TAs > thr2) && (lane <= last_lane));
          const int lstar = m ? (int)__builtin_ctzll(m) : last_lane;
          const float E = lstar > 0 ? readlane_f(TAs, lstar - 1) : 0.0f;
          int jsel = 0;
          if (lane == lstar) {
            float a = 0.0f;
            int cnt = 0;
#pragma unroll
            for (int j = 0; j < C; ++j) {
              a = __builtin_fmaf(coef[lane * C + j], beta, a);
              cnt += (E + a <= thr2) ? 1 : 0;
            }
            jsel = cnt < C ? cnt : last_j;
          }
          kn = lstar * C + readlane_i(jsel, lstar);
        }

        if (p.trace != nullptr && lane == 0) {
          float* tr = p.trace + 8 * t;
          tr[0] = (float)kn;
          tr[1] = sumB;
          tr[2] = sumA;
          tr[3] = thr;
          tr[4] = (float)n;
          tr[5] = (float)zo;
          tr[6] = (float)w;
          tr[7] = u;
        }
        // add the token back under its new topic
        {
          const int ndk = nd[kn] + 1;
          if (lane == 0) nd[kn] = ndk;
          wave_lds_fence();
          const int ndz = (kn == zo) ? ndk : nd[zo];
          const float cfz = ((float)ndz + t_alpha[zo]) * t_inv[zo];
          const float cfk = ((float)ndk + t_alpha[kn]) * t_inv[kn];
          if (lane == 0) {
            coef[zo] = cfz;
            coef[kn] = cfk;
          }
          wave_lds_fence();
          if (lane == lo || lane == kn / C) TA = coef_partial<C>(coef + lane * C, beta);
        }
        cn = (lane == idx) ? kn : cn;
        if (!FROZEN && kn != zo) {
          if (lane < 2) {
            const int k = lane == 0 ? zo : kn;
            const int v = lane == 0 ? -1 : 1;
            atomicAdd(&p.delta[(int64_t)w * KP + k], v);
            atomicAdd(&bsum[k], v);
          }
        }

        // keep the pipeline full: first R0 rounds of token t+P
        const int64_t tp = t + P;
        if (tp < t1) {
          const int pidx = (int)(tp - cbase);
          int np;
          int64_t op;
          if (pidx < 64) {
            np = readlane_i(cmn, pidx) & 0x7FFFFFFF;
            op = ((int64_t)readlane_i((int)(cmo >> 32), pidx) << 32) | (uint32_t)readlane_i((int)cmo, pidx);
          } else {
            np = readlane_i(m1n, pidx - 64) & 0x7FFFFFFF;
            op = ((int64_t)readlane_i((int)(m1o >> 32), pidx - 64) << 32) |
                 (uint32_t)readlane_i((int)m1o, pidx - 64);
          }
#pragma unroll
          for (int q = 0; q < R0; ++q) ring[s][q] = (q * 64 + lane < np) ? ent[op + q * 64 + lane] : 0u;
        }
      }
    }
    if (cbase + lane < t1) p.z[cbase + lane] = cn;
#pragma unroll
    for (int j = 0; j < C; ++j) nd[lane * C + j] = 0;
    wave_lds_fence();
  }

  if (!FROZEN && p.dsum) {
    __syncthreads();
    for (int i = threadIdx.x; i < KP; i += 256) {
      const int v = bsum[i];
      if (v != 0) atomicAdd(&p.dsum[i], v);
    }
  }
}

// ------------------------------------------- the large-K sparse sampler
// K up to 4096 (C = 32, 64), round 5 (v9).  The draw (oracle/lda_oracle.c:
// exact_draw_big) splits p_k = (nd_k + a_k)(nw_k + b) inv_k into
//   B, the word part, over the word's nonzero entries (lane l holds entries
//     l, l+64, ...): coef_t = fma(nd_t, inv_t, ainv_t), acc = fma(c, coef, acc)
//     -- one fma chain per entry and no own-token test per entry: the
//     token's own entry enters B uncorrected and is corrected afterwards by
//     an exact accept / re-draw step (below);
//   A, the doc part beta * sum_k (nd_k + a_k) inv'_k, held EXACTLY as a
//     64-bit fixed-point sum: sum_k G'_k (per sweep, k_big_tables) plus
//     R = sum_k nd_k F_k, which a token updates with two integer adds (the
//     previous token's new topic in, this token's old topic out).
// So a token's fixed work is a handful of scalar-ish operations where v8
// re-evaluated and re-scanned three 16-topic groups of the doc part per token
// (~60 VALU), and a word entry costs ~8 VALU + 2 LDS reads instead of ~14.
//
// The own token.  B holds its entry as x = c * coef_zo; the exact weight of
// that entry is O = (c - 1) * fma(nd_zo, inv_m1_zo, ainv_m1_zo) <= x (c <=
// nwsum).  A draw that lands in the entry keeps zo with probability O / w
// (w = the entry's width in its lane's running sums); otherwise the draw is
// repeated once over the same sums with the entry's width replaced by O
// (the second uniform mapped around the entry).  Together that is exactly
// the corrected distribution; only draws that hit the own entry pay for it.
//
// Work distribution and LDS are v8's: 16-wave blocks, a block-wide float2
// {inv, ainv} table and per-wave 16-bit document counts (documents < 65536
// tokens).  The word part streams rounds of 64 entries: the first RB rounds
// of the next tokens sit in a ring of NS slots (refilled right after a token
// has used its own rounds, so every wait covers loads issued at least one
// token earlier), as bounded buffer loads whose range ends at the row's last
// entry: the zero padding of a row's last round (k_build_sparse) is never
// fetched.  Count changes go out per 64-token chunk (lane i: token i).
#ifndef SB_RB
#define SB_RB 12
#endif
#ifndef SB_NS
#define SB_NS 2
#endif
#ifndef SB_RB_SHORT
#define SB_RB_SHORT 6
#endif
#ifndef SB_NS_SHORT
#define SB_NS_SHORT 4
#endif
// rows past the register rounds: batches of SB_BATCH rounds, double-buffered;
// each lane keeps its running sum after each of the first SB_NB batches so a
// draw in a long row re-reads one batch of the selected lane
#ifndef SB_BATCH
#define SB_BATCH 4
#endif
#ifndef SB_NB
#define SB_NB 2
#endif
// 1: the ring refill of token t+NS-1 issued last in token t, after the
// long-row batches and the draw's rare paths, whose loads are waited for
// right after they are issued (in-order vmcnt: such a wait drains every older
// load, the refill included when it was issued before them)
#ifndef SB_REFILL_LAST
#define SB_REFILL_LAST 0
#endif
// register rounds evaluated without a branch (the rest: one uniform branch
// each); they share a basic block with the doc part's fixed-point chain
#ifndef SB_RU
#define SB_RU 2
#endif
// 1 (default since round 6): the A part's searches read LDS (the alpha
// part's block from tab, the document part's per-lane sums with rotated
// reads) instead of global memory -- one global round trip instead of two and
// eight.  Same integers either way: 32 large-K parity tests green on both
// builds; C5 2.18 -> 2.29e9 near init, 2.70 -> 2.77e9 after 30 sweeps
// (profiles/r06/c5ab/).  0 keeps round 5's global-memory searches.
#ifndef SB_APICK_LDS
#define SB_APICK_LDS 1
#endif
// > 0 (default 4 since late round 6): the LDS reads (tab + document count)
// of the first SB_LDS_BATCH register rounds are all issued, with the doc
// part's, before the first is used -- one LDS round trip for those rounds
// instead of one per round (the compiler had serialised them: one pair of
// reads, wait, fma, the next pair); the sums are the same fma for fma.
// SB_LDS_BATCH2 > 0: the next SB_LDS_BATCH2 rounds the same way, when the
// row has them.  C5 with SB_TOKEN_LGKM0 (below), one session, both orders
// (profiles/r06/ldsbatch/): near init 2.250 -> 2.294e9, after 30 sweeps
// 2.730 -> 2.828e9; batches of 6 or all 12 rounds gain less.
#ifndef SB_LDS_BATCH
#define SB_LDS_BATCH 4
#endif
#ifndef SB_LDS_BATCH2
#define SB_LDS_BATCH2 0
#endif
#ifndef SB_LDS_BATCH_ADDR
#define SB_LDS_BATCH_ADDR 0
#endif
// 1 (default since late round 6): an lgkmcnt(0) at the end of every token,
// where every LDS read of the token has been used anyway: without it the
// waitcnt pass carried a rare path's pending LDS write across the loop's
// join into the next token, as an lgkmcnt(0) between the batch's first reads
// and the rest
#ifndef SB_TOKEN_LGKM0
#define SB_TOKEN_LGKM0 1
#endif
// 1 (A/B builds): the long rows' batches past the register rounds issue each
// batch's LDS reads together as well
#ifndef SB_LDS_BATCH_LONG
#define SB_LDS_BATCH_LONG 0
#endif
// gfx9 buffer resource word 3 (raw 32-bit loads, bounds checked)
constexpr int kBufWord3 = 0x00020000;
#ifndef SB_WAVES
#define SB_WAVES 16
#endif
template <int C>
constexpr int sb_waves() { return SB_WAVES; }

// Philox words x0, x1, x2 of a token's block, lane-parallel per 64-token
// chunk (the large-K draw: x0 the draw, x1 the own-entry accept test, x2 the
// rare re-draw; computed per token inside the re-draw branch, the compiler
// hoisted the whole block into every token's scalar path)
__device__ __forceinline__ void philox_x012(uint64_t gtok, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                            uint32_t& x0, uint32_t& x1, uint32_t& x2) {
  uint32_t c0 = (uint32_t)gtok, c1 = (uint32_t)(gtok >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r > 0) {
      k0 += PHILOX_W0;
      k1 += PHILOX_W1;
    }
    const uint32_t hi0 = __umulhi(PHILOX_M0, c0), lo0 = PHILOX_M0 * c0;
    const uint32_t hi1 = __umulhi(PHILOX_M1, c2), lo1 = PHILOX_M1 * c2;
    const uint32_t n0 = hi1 ^ c1 ^ k0;
    const uint32_t n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
  }
  x0 = c0;
  x1 = c1;
  x2 = c2;
}
__device__ __forceinline__ void philox_x01(uint64_t gtok, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1,
                                           uint32_t& x0, uint32_t& x1) {
  uint32_t x2;
  philox_x012(gtok, c2, c3, k0, k1, x0, x1, x2);
}
__device__ __forceinline__ float uniform_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// floor(x) for 0 <= x < 2^64 (C's (uint64_t)x): both conversions truncate,
// x - hi 2^32 is exact
__device__ __forceinline__ uint64_t d2u64(double x) {
  const uint32_t hi = (uint32_t)(x * 0x1p-32);
  const uint32_t lo = (uint32_t)(x - (double)hi * 0x1p32);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) { return (uint64_t)uniform_l((int64_t)v); }
__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d) {
  const int lane = threadIdx.x & 63;
  const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, lane - d < 0 ? lane : lane - d);
  const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), lane - d < 0 ? lane : lane - d);
  return lane >= d ? (((uint64_t)hi << 32) | lo) : 0ull;
}
// inclusive wave scan of 64-bit integers (exact in any order)
__device__ __forceinline__ uint64_t wave_incl_scan_u64(uint64_t v) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) v += shfl_up_u64(v, d);
  return v;
}
__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, o);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), o);
    v += ((uint64_t)hi << 32) | lo;
  }
  return v;
}

// Per-sweep tables of the large-K draw (oracle exact_big_tables), one block
// of 1024 threads (Kp <= 4096): m = the largest table value (inv, ainv and,
// for topics holding tokens, inv_m1, ainv_m1), S = 31 - exponent(m), the
// fixed-point values big_fix(x) = (uint32) ldexp(x, S) < 2^31, the prefix of
// G = big_fix(ainv) and the scalars bsig = beta 2^-S, isig = 2^S / beta.
__device__ __forceinline__ uint32_t big_fix(float x, int S) { return (uint32_t)ldexpf(x, S); }

__global__ __launch_bounds__(1024) void k_big_tables(const int32_t* __restrict__ nwsum,
                                                     const float* __restrict__ alpha_f,
                                                     const float* __restrict__ inv,
                                                     const float* __restrict__ inv_m1, int32_t K, int32_t Kp,
                                                     float beta, BigTables t) {
  __shared__ float smax[16];
  __shared__ uint64_t ssum[1024];
  const int tid = threadIdx.x;
  const int per = (Kp + 1023) / 1024;   // <= 4
  float m = 0.0f;
  float vi[4], va[4], vim[4], vam[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = tid * per + j;
    vi[j] = va[j] = vim[j] = vam[j] = 0.0f;
    if (j >= per || k >= Kp) continue;
    const bool live = k < K && nwsum[k] >= 1;
    vi[j] = inv[k];
    va[j] = alpha_f[k] * vi[j];
    vim[j] = live ? inv_m1[k] : 0.0f;
    vam[j] = live ? alpha_f[k] * inv_m1[k] : 0.0f;
    t.tab[k] = make_float2(vi[j], va[j]);
    m = fmaxf(m, fmaxf(fmaxf(vi[j], va[j]), fmaxf(vim[j], vam[j])));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((tid & 63) == 0) smax[tid >> 6] = m;
  __syncthreads();
  float mm = 0.0f;
#pragma unroll
  for (int i = 0; i < 16; ++i) mm = fmaxf(mm, smax[i]);
  int e = 0;
  (void)frexpf(mm, &e);
  const int S = mm > 0.0f ? 31 - e : 0;
  uint64_t loc = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = tid * per + j;
    if (j >= per || k >= Kp) continue;
    const uint32_t G = big_fix(va[j], S);
    t.F[k] = big_fix(vi[j], S);
    t.tab_m1[k] = make_float4(vim[j], vam[j], __builtin_bit_cast(float, big_fix(vim[j], S)),
                              __builtin_bit_cast(float, (int32_t)big_fix(vam[j], S) - (int32_t)G));
    loc += G;
  }
  ssum[tid] = loc;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {
    const uint64_t v = tid >= d ? ssum[tid - d] : 0ull;
    __syncthreads();
    ssum[tid] += v;
    __syncthreads();
  }
  uint64_t acc = ssum[tid] - loc;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = tid * per + j;
    if (j >= per || k >= Kp) continue;
    acc += big_fix(va[j], S);
    t.pfx[k] = acc;
  }
  if (tid == 0) {
    BigScal s;
    s.S = S;
    s.pad = 0;
    s.S0 = ssum[1023];
    s.bsig = ldexpf(beta, -S);
    s.bsig_hi = ldexpf(beta, 32 - S);
    s.isig = ldexp(1.0, S) / (double)beta;
    *t.scal = s;
  }
}

// Inclusive integer wavefront scan (any order is exact for integers).
__device__ __forceinline__ int wave_incl_scan_i(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, true);
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);
  return x;
}

// SB_ND8 (measurement builds, round 6): the per-wave document counts as
// bytes (documents of at most 255 tokens of one topic), 4 KiB per wave at
// K = 4096 instead of 8 KiB, so that two 10-wave blocks (20 waves per CU,
// with SB_WAVES 10 and SB_WPE 5) fit the 160 KiB of LDS
#ifndef SB_ND8
#define SB_ND8 0
#endif
#ifndef SB_WPE
#define SB_WPE 0
#endif
#if SB_ND8 && !SB_APICK_LDS
#error "SB_ND8 needs SB_APICK_LDS (the global-memory doc search reads 16-bit pairs)"
#endif
constexpr int kNdShift = SB_ND8 ? 2 : 1;     // counts per 32-bit LDS word: 4 or 2
constexpr int kNdBits = SB_ND8 ? 8 : 16;
__device__ __forceinline__ int nd16_get(const uint32_t* nd2, int k) {
#if SB_ND8
  return (int)reinterpret_cast<const uint8_t*>(nd2)[k];
#endif
  return (int)reinterpret_cast<const uint16_t*>(nd2)[k];
}

// A SampleParams field read from the kernel-argument segment where it is used
// (the kernel's only argument sits at offset 0).  The large-K sampler runs
// out of SGPRs (36 spilled into VGPR lanes with every pointer held live);
// pointers of rare paths (chunk and document switches, the doc-part search,
// saturated rows) are re-read from the segment instead of held.
// SB_X_COUNT (measurement builds only): per-path draw counters in p.trace
// ([0] tokens, [1] A alpha part, [2] A doc part, [3] own-entry hits, [4]
// re-draws) when the launch has a trace buffer (lda_debug_sample_trace;
// plain sweeps have none)
#ifdef SB_X_COUNT
#define SB_COUNT(i)                                                                   \
  do {                                                                                \
    unsigned* ct_ = reinterpret_cast<unsigned*>(KARG(trace));                      \
    if ((threadIdx.x & 63) == 0 && ct_ != nullptr) atomicAdd(ct_ + (i), 1u);       \
  } while (0)
#else
#define SB_COUNT(i) \
  do {              \
  } while (0)
#endif
// SB_GLOBAL_AS: the pointers a KARG read yields are used as global (address
// space 1) pointers (KGLOBAL), so the count atomics are global_atomic, not
// FLAT.  A FLAT operation still in flight (the no-return delta atomics of a
// chunk switch) makes the waitcnt pass order every later vector memory wait
// as vmcnt(0); merged into the loop's join, that had drained the ring of
// prefetched rows at every token's first round (now vmcnt(14..19)).  2 (the
// default since late round 6): the field itself still read as a FLAT load,
// waited for where it is used.  1 (A/B): the field read through the kernarg
// segment's address space -- scalar loads, 7% slower on C5.  0: round 5's
// FLAT atomics.  C5, four sessions: +0.2-0.5% near init, +0.4-0.7% after
// burn-in (profiles/r06/ldsbatch/r6v, r6w).
#ifndef SB_GLOBAL_AS
#define SB_GLOBAL_AS 2
#endif
// 1: the chunk switch waits vmcnt(1) for its chunk registers (round 4: with
// FLAT atomics in flight the waitcnt pass had turned every later wait into
// vmcnt(0)); 0 (A/B) leaves the waits to the compiler
// 1 (default since late round 6): the alpha part's 64 block-end prefixes
// (fixed for the sweep) in a register pair per lane for the whole launch
// instead of one global round trip per A-alpha draw (8.7% of the draws).  Two
// VGPRs spill in the 4 x 6 ring; still C5 +1.1-1.3% near init, +0.9% after
// burn-in, two sessions (profiles/r06/ldsbatch/r6y)
#ifndef SB_PFX_REG
#define SB_PFX_REG 1
#endif
// 1 (default since late round 6): the A search's document part sums only the
// nonzero count words of each lane's block (a mask first), not all C topics:
// the same integers; C5 +0.5-0.7% near init, flat after burn-in
// (profiles/r06/ldsbatch/r6z)
#ifndef SB_ADOC_SPARSE
#define SB_ADOC_SPARSE 1
#endif
// 1 (default since late round 6): a long row's first batch past the register
// rounds loaded at the token's start instead of after the rounds, so its
// memory latency overlaps them; C5 +2.7% near init, +1.5% after burn-in, two
// sessions (profiles/r06/ldsbatch/r6ac, r6ad).  2 (the second batch too)
// spills 6 VGPRs and loses.
#ifndef SB_EARLY_BATCH
#define SB_EARLY_BATCH 1
#endif
// 1 (default since late round 6): the ring slot of token t-1 refilled at
// token t's start rather than after t's register rounds -- possible once no
// FLAT operation forces vmcnt(0) (SB_GLOBAL_AS): C5 after 30 sweeps +1.3%,
// near init within noise, two sessions (profiles/r06/ldsbatch/r6af)
#ifndef SB_REFILL_FIRST
#define SB_REFILL_FIRST 1
#endif
// 1 (A/B): Philox x1 (the own-entry accept test) computed on the own-entry
// path instead of held per lane for the chunk (one VGPR)
#ifndef SB_X1_LAZY
#define SB_X1_LAZY 0
#endif
// 1 (default at the end of round 6): a new document's counts built from the
// chunk registers instead of a memory read of its topics; the same counts,
// C5 +0.3% after burn-in, flat near init (profiles/r06/ldsbatch/r6am)
#ifndef SB_DOC_REGS
#define SB_DOC_REGS 1
#endif
#ifndef SB_CHUNK_WAIT
#define SB_CHUNK_WAIT 1
#endif
#if SB_GLOBAL_AS
#if SB_GLOBAL_AS == 1
#define KARG(field)                                                                                   \
  (*(const volatile __attribute__((address_space(4))) decltype(SampleParams::field)*)(                 \
      (const __attribute__((address_space(4))) char*)(__builtin_amdgcn_kernarg_segment_ptr()) +        \
      offsetof(SampleParams, field)))
#else
// 2: the field read as before (a FLAT load, waited for where it is used),
// only the pointers' own accesses global
#define KARG(field)                                                                                   \
  (*reinterpret_cast<const volatile decltype(SampleParams::field)*>(                                  \
      (const char*)(__builtin_amdgcn_kernarg_segment_ptr()) + offsetof(SampleParams, field)))
#endif
template <typename T>
__device__ __forceinline__ __attribute__((address_space(1))) T* kglobal(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}
template <typename T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* kglobal(const T* p) {
  return (const __attribute__((address_space(1))) T*)p;
}
#define KGLOBAL(field) kglobal(KARG(field))
#define KATOMIC_ADD(ptr, v) __hip_atomic_fetch_add((ptr), (v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
#else
#define KARG(field)                                                                                   \
  (*reinterpret_cast<const volatile decltype(SampleParams::field)*>(                                  \
      (const char*)(__builtin_amdgcn_kernarg_segment_ptr()) + offsetof(SampleParams, field)))
#define KGLOBAL(field) KARG(field)
#define KATOMIC_ADD(ptr, v) atomicAdd((ptr), (v))
#endif
template <int C, int NS, int RB, bool FROZEN>
#if SB_WPE
#define SB_ATTR __attribute__((amdgpu_waves_per_eu(SB_WPE, SB_WPE)))
#else
#define SB_ATTR
#endif
__global__ __launch_bounds__(64 * sb_waves<C>()) SB_ATTR void k_sample_big(SampleParams p) {
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  constexpr int KP = C * 64;
  constexpr int WB = sb_waves<C>();
  static_assert(NS >= 2 && NS <= 8, "ring slots");
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float2* tab = reinterpret_cast<float2*>(smem);                              // [KP] {inv, ainv}
  constexpr int NDW = KP >> kNdShift;                                          // LDS words of a wave's counts
  uint32_t* nd2 = reinterpret_cast<uint32_t*>(smem + 2 * KP) + wid * NDW;      // [KP/2] (16-bit) or [KP/4]

  for (int i = threadIdx.x; i < KP; i += 64 * WB) tab[i] = p.big.tab[i];
  for (int i = threadIdx.x; i < WB * NDW; i += 64 * WB) smem[2 * KP + i] = 0;
  __syncthreads();

  const int S = uniform_i(p.big.scal->S);
  const uint64_t S0 = uniform_u64(p.big.scal->S0);
  const float bsig = p.big.scal->bsig, bsig_hi = p.big.scal->bsig_hi;
  const double isig = p.big.scal->isig;
  const int last_topic = p.K - 1;
  const uint32_t* __restrict__ ent = p.ent;
  const uint32_t* __restrict__ row_off = p.row_rnd;   // a row's start in whole 64-entry rounds
  auto row_ptr = [&](uint32_t o) -> const uint32_t* { return ent + ((uint64_t)o << 6); };
  const int32_t* __restrict__ row_nnz = p.row_nnz;
  const float4* __restrict__ tab_m1 = p.big.tab_m1;
#if SB_PFX_REG
  // the alpha part's block-end prefixes (fixed for the sweep) held per lane:
  // the A search's block choice without a global round trip
  const uint64_t pfx_r = p.big.pfx[C * lane + C - 1];
#endif

  auto fixp = [&](float x) -> uint32_t { return big_fix(x, S); };
  // one B term into the lane's running sum (SAT: the row holds a saturated
  // count field, read the exact count from nw)
  auto term_acc = [&](uint32_t e, int w, bool sat, float acc) -> float {
    const int t = (int)(e & ENT_TOPIC_MASK);
    uint32_t c = e >> ENT_TOPIC_BITS;
    if (sat && c == ENT_COUNT_SAT) c = (uint32_t)KGLOBAL(nw)[(int64_t)w * KP + t];
    const float2 tb = tab[t];
    const float coef = __builtin_fmaf((float)nd16_get(nd2, t), tb.x, tb.y);
    return __builtin_fmaf((float)c, coef, acc);
  };
  // the pieces of a term (re-walks of a batch by readlane)
  auto term_parts = [&](uint32_t e, int w, bool sat, float& cf, float& coef) {
    const int t = (int)(e & ENT_TOPIC_MASK);
    uint32_t c = e >> ENT_TOPIC_BITS;
    if (sat && c == ENT_COUNT_SAT) c = (uint32_t)KGLOBAL(nw)[(int64_t)w * KP + t];
    const float2 tb = tab[t];
    coef = __builtin_fmaf((float)nd16_get(nd2, t), tb.x, tb.y);
    cf = (float)c;
  };

  bool first_range = true;
  while (true) {
    int r = 0;
    if ((!LDA_STATIC_FIRST || !first_range) && lane == 0) r = atomicAdd(p.queue, 1);
    r = uniform_i(first_or_queued(first_range, (int)blockIdx.x * WB + wid, (int)gridDim.x * WB, uniform_i(__shfl(r, 0))));
    first_range = false;
    if (r >= p.num_ranges) break;
    const int64_t d0 = p.range_doc[r], d1 = p.range_end[r];
    const int64_t t0 = p.doc_off[d0];
    const int t1 = (int)(p.doc_off[d1] - t0);
    if (t1 <= 0) continue;
    const int32_t* __restrict__ wrd = p.words + t0;
    int32_t* __restrict__ zr = p.z + t0;
    const uint64_t gbase = (uint64_t)(p.token_base + t0);

    int cbase = 0;
    int cw = 0, cz = 0, w1 = 0, z1 = 0, w2 = 0, z2 = 0;
    if (lane < t1) {
      cw = wrd[lane];
      cz = zr[lane];
    }
    if (64 + lane < t1) {
      w1 = wrd[64 + lane];
      z1 = zr[64 + lane];
    }
    if (128 + lane < t1) {
      w2 = wrd[128 + lane];
      z2 = zr[128 + lane];
    }
    int cmn = row_nnz[cw], m1n = row_nnz[w1];
    uint32_t cmo = row_off[cw], m1o = row_off[w1];
    int cn = cz;
    uint32_t cx0, cx1;
    philox_x01(gbase + (uint64_t)lane, p.c2, p.c3, p.k0, p.k1, cx0, cx1);
    __builtin_amdgcn_s_waitcnt(kVmcnt0);

    // SB_X_NODELTA: attribution builds only (wrong counts): no delta atomics.
    // Not informative as run in round 6: without the changes the counts stay
    // at their random start, the rows stay long and the sweep ran 2x slower.
    // SB_X_DELTA_KERNEL: the same sampler with the count changes made right
    // by k_delta_from_z after it (lda_capi.cpp), an A/B of where the atomics
    // cost less (measurement builds only)
#if defined(SB_X_NODELTA) || defined(SB_X_DELTA_KERNEL)
    constexpr bool kDelta = false;
#else
    constexpr bool kDelta = !FROZEN;
#endif
    auto flush_chunk = [&]() {
      if (kDelta && cn != cz) {
        const uint64_t rb = (uint64_t)(uint32_t)cw * (uint64_t)KP;
        KATOMIC_ADD(KGLOBAL(delta) + (rb + (uint32_t)cz), -1);
        KATOMIC_ADD(KGLOBAL(delta) + (rb + (uint32_t)cn), 1);
      }
    };

    // document start: counts into LDS, R = sum of F over the document's topics
    uint64_t R = 0;
    auto build_doc = [&](int ts, int te) {
      uint64_t rl = 0;
      auto add_topic = [&](int k) {
#if SB_ND8
        atomicAdd(&nd2[k >> 2], 1u << (8 * (k & 3)));
#else
        atomicAdd(&nd2[k >> 1], (k & 1) ? 0x10000u : 1u);
#endif
        rl += fixp(tab[k].x);
      };
#if SB_DOC_REGS
      // the document's topics from the chunk registers (tokens cbase ..
      // cbase + 191, not yet sampled: their old topics, as z in memory
      // holds them), memory only past them -- no load on a document switch
      // of a document that fits
      {
        const int i0 = cbase + lane;
        if (i0 >= ts && i0 < te) add_topic(cz);
        if (i0 + 64 >= ts && i0 + 64 < te) add_topic(z1);
        if (i0 + 128 >= ts && i0 + 128 < te) add_topic(z2);
      }
      for (int i = (ts > cbase + 192 ? ts : cbase + 192) + lane; i < te; i += 64) add_topic(zr[i]);
#else
      for (int i = ts + lane; i < te; i += 64) add_topic(zr[i]);
#endif
      R = uniform_u64(wave_sum_u64(rl));
      wave_lds_fence();
    };
    auto clear_doc = [&]() {
#pragma unroll
      for (int j = 0; j < NDW / 64; j += 4)
        *reinterpret_cast<uint4*>(nd2 + lane * (NDW / 64) + j) = make_uint4(0u, 0u, 0u, 0u);
      wave_lds_fence();
    };

    int64_t doc = d0;
    while (p.doc_off[doc + 1] <= t0) ++doc;
    int doc_end = uniform_i((int)(p.doc_off[doc + 1] - t0));
    build_doc(0, doc_end);

    // ring slot of token t: t % NS; slot (t + NS - 1) % NS is refilled during t
    // the ring and the running sums as register vectors: the draw indexes
    // them by a wave-uniform round (an indexed register move; as arrays they
    // were placed in scratch)
    typedef uint32_t ring_t __attribute__((ext_vector_type(RB)));
    typedef float accq_t __attribute__((ext_vector_type(RB)));
    ring_t ring[NS];
    // per slot, the token's old topic: {inv_m1, ainv_m1, bits of Fm1, bits
    // of Gm1 - G} (k_big_tables), loaded FIRST so the doc part can be formed
    // at the token's start, off the draw's chain
    float4 rm1[NS];
    auto prefetch = [&](ring_t& rg, float4& m1, int tp) {
      const int pidx = tp - cbase;
      int np, zp;
      uint32_t op;
      if (pidx < 64) {
        np = readlane_i(cmn, pidx);
        op = (uint32_t)readlane_i((int)cmo, pidx);
        zp = readlane_i(cz, pidx);
      } else {
        np = readlane_i(m1n, pidx - 64);
        op = (uint32_t)readlane_i((int)m1o, pidx - 64);
        zp = readlane_i(z1, pidx - 64);
      }
      if (!FROZEN) m1 = tab_m1[zp];
      // the range ends at the row's last entry: loads past it (the zero
      // padding of the last round, rounds past the row, tokens past the
      // range) return 0 without a memory access
      const int nb = tp < t1 ? (np & 0x7FFFFFFF) * 4 : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)row_ptr(op), (short)0, nb, kBufWord3);
      // lane * 4 opaque here: the constant q * 256 then folds into the loads'
      // immediate offset (hoisted out of the loop, lane * 4 + q * 256 had
      // taken one VGPR per round)
      int lo4 = lane * 4;
      asm volatile("" : "+v"(lo4));
#pragma unroll
      for (int q = 0; q < RB; ++q) rg[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, lo4 + q * 256, 0, 0);
    };
#pragma unroll
    for (int s = 0; s < NS - 1; ++s) prefetch(ring[s], rm1[s], s);

    int pk = -1;   // the previous token of this document: its new topic, still to add back
    for (int tb = 0; tb < t1; tb += NS) {
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int t = tb + s;
        if (t < t1) {
          int idx = t - cbase;
          if (idx == 64) {
            // the finished chunk's topics and count changes
            const int ow = cw, oz = cz, on = cn;
            const int ob = cbase;
            cbase += 64;
            idx = 0;
            cw = w1;
            cz = z1;
            cmn = m1n;
            cmo = m1o;
            w1 = w2;
            z1 = z2;
            m1n = row_nnz[w1];
            m1o = row_off[w1];
            cn = cz;
            if (cbase + 128 + lane < t1) {
              w2 = wrd[cbase + 128 + lane];
              z2 = zr[cbase + 128 + lane];
            }
            zr[ob + lane] = on;
            // the chunk registers land here, once per 64 tokens (every load
            // but the z store just issued): a chunk register the compiler
            // believes in flight makes it wait vmcnt(0) where a token reads
            // it, i.e. drain the row ring
#if SB_CHUNK_WAIT
            __builtin_amdgcn_s_waitcnt(kVmcnt1);
#endif
            if (kDelta && on != oz) {
              const uint64_t rb = (uint64_t)(uint32_t)ow * (uint64_t)KP;
              KATOMIC_ADD(KGLOBAL(delta) + (rb + (uint32_t)oz), -1);
              KATOMIC_ADD(KGLOBAL(delta) + (rb + (uint32_t)on), 1);
            }
            philox_x01(gbase + (uint64_t)(cbase + lane), p.c2, p.c3, p.k0, p.k1, cx0, cx1);
          }
          if (t == doc_end) {
            clear_doc();
            ++doc;
            const auto dof = KGLOBAL(doc_off);
            while (dof[doc + 1] - t0 <= t) ++doc;
            doc_end = uniform_i((int)(dof[doc + 1] - t0));
            build_doc(t, doc_end);
            pk = -1;
          }

#if SB_REFILL_FIRST
          {
            // the slot of token t-1 refilled first thing (its registers were
            // used up by token t-1): with no FLAT operation in flight the
            // waits for this token's own slot count past these loads
            // (vmcnt(N)), and the next rows get a fuller token of lead
            const int sp = (s + NS - 1) % NS;
            prefetch(ring[sp], rm1[sp], t + NS - 1);
          }
#endif
          const int w = readlane_i(cw, idx);
          const int zo = readlane_i(cz, idx);
          const float u = u01((uint32_t)readlane_i((int)cx0, idx));
          const int n_raw = readlane_i(cmn, idx);
          const bool row_sat = n_raw < 0;
          const int n = n_raw & 0x7FFFFFFF;
          const uint32_t off = (uint32_t)readlane_i((int)cmo, idx);
          const uint32_t* __restrict__ erow = row_ptr(off);

          // the previous token back under its new topic, this one out: two
          // LDS adds in flight at once; the old count comes back for the
          // fixed-point own-topic terms
          if (lane == 0) {
            const int pa = pk >= 0 ? pk : 0;
#if SB_ND8
            __hip_atomic_fetch_add(&nd2[pa >> 2], pk < 0 ? 0u : (1u << (8 * (pa & 3))), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_add(&nd2[zo >> 2], 0xFFFFFFFFu << (8 * (zo & 3)), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
#else
            __hip_atomic_fetch_add(&nd2[pa >> 1], pk < 0 ? 0u : ((pa & 1) ? 0x10000u : 1u), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
            __hip_atomic_fetch_add(&nd2[zo >> 1], (zo & 1) ? 0xFFFF0000u : 0xFFFFFFFFu, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WAVEFRONT);
#endif
          }
          wave_lds_fence();
          // the own topic's count after both updates (a plain read behind the
          // no-return adds: a wave's LDS operations complete in order; a
          // returning atomic held the rounds' reads behind it) and R's update
          // are formed in doc_part, in the basic block of the first rounds:
          // formed here, ahead of the row_sat branch, their reads were waited
          // for (lgkmcnt(0)) before the rounds' reads were even issued
          int ndz = 0;
          uint32_t Fz = 0;

          // word part, register rounds: lane l holds entry l + 64 q; accq[q]
          // = the lane's running sum after round q
          const int nr_all = (n + 63) >> 6;
          accq_t accq;
          float acc = 0.0f;
          // the doc part, A_fx = sum_k nd_k F'_k + sum_k G'_k (exact), from
          // the slot's topic data; written out in the same basic block as the
          // first SB_RU rounds (evaluated without a branch: a round past the
          // row is zero entries, + 0), so the scheduler interleaves the two
          // chains.  A row holding a saturated count takes the general path.
          int64_t dG = 0;
          uint32_t Fm1z = 0;
          uint64_t As = S0;
          float A_f = 0.0f;
          // its LDS reads first in the block (issued with, and ahead of, the
          // rounds' reads: one LDS round trip for both), the rest after the
          // first rounds
          struct DocReads {
            int nz;
            float iz, ip;
          };
          auto doc_reads = [&]() __attribute__((always_inline)) -> DocReads {
            return DocReads{nd16_get(nd2, zo), tab[zo].x, tab[pk >= 0 ? pk : 0].x};
          };
          auto doc_part = [&](const DocReads dr) __attribute__((always_inline)) {
            ndz = uniform_i(dr.nz);
            Fz = (uint32_t)uniform_i((int)fixp(dr.iz));
            const float2 tp = make_float2(dr.ip, 0.0f);
            // (a mask, not a branch: the read stays beside the others)
            const uint32_t Fp = (uint32_t)uniform_i((int)fixp(tp.x)) & (uint32_t)(-(int)(pk >= 0));
            R = R + (uint64_t)Fp - (uint64_t)Fz;
            uint64_t Afx;
            if (!FROZEN) {
              const float4 m1 = rm1[s];
              Fm1z = (uint32_t)uniform_i(__builtin_bit_cast(int, m1.z));
              dG = (int64_t)uniform_i(__builtin_bit_cast(int, m1.w));
              const int64_t dF = (int64_t)ndz * ((int64_t)Fm1z - (int64_t)Fz);
              As = (uint64_t)((int64_t)S0 + dG);
              Afx = (uint64_t)((int64_t)(As + R) + dF);
            } else {
              Afx = S0 + R;
            }
            // A in fp32: beta 2^-S (hi 2^32 + lo), hi < 2^16 exact
#ifdef SB_X_NOA
            A_f = uniform_f((float)(uint32_t)S0 * bsig);   // attribution experiment only
            (void)Afx;
#else
            A_f = uniform_f(__builtin_fmaf((float)(uint32_t)uniform_i((int)(uint32_t)(Afx >> 32)), bsig_hi,
                                           (float)(uint32_t)uniform_i((int)(uint32_t)Afx) * bsig));
#endif
          };
          auto rounds = [&](bool sat, int q0) __attribute__((always_inline)) {
#pragma unroll
            for (int q = 0; q < RB; ++q) {
              if (q < q0) continue;
              if (q < nr_all) acc = term_acc(ring[s][q], w, sat, acc);
              accq[q] = acc;
            }
          };
          // (the memory barriers keep the doc reads in the branches: hoisted
          // above the branch, their wait and conversions went with them)
#if SB_EARLY_BATCH
          // a long row's first batch past the register rounds issued now, so
          // its latency overlaps the rounds (zeros when the row has none)
          uint32_t ea0[SB_BATCH];
#if SB_EARLY_BATCH >= 2
          uint32_t eb0[SB_BATCH];
#endif
          {
            const __amdgpu_buffer_rsrc_t rb0 = __builtin_amdgcn_make_buffer_rsrc(
                (void*)erow, (short)0, nr_all > RB ? n * 4 : 0, kBufWord3);
            int lo4 = lane * 4;
            asm volatile("" : "+v"(lo4));
#pragma unroll
            for (int b = 0; b < SB_BATCH; ++b) ea0[b] = __builtin_amdgcn_raw_buffer_load_b32(rb0, lo4 + (RB + b) * 256, 0, 0);
#if SB_EARLY_BATCH >= 2
            // and the second (a row shorter than it reads zeros: the bound
            // is the row's own length)
#pragma unroll
            for (int b = 0; b < SB_BATCH; ++b)
              eb0[b] = __builtin_amdgcn_raw_buffer_load_b32(rb0, lo4 + (RB + SB_BATCH + b) * 256, 0, 0);
#endif
          }
#endif
          if (!row_sat) {
            asm volatile("" ::: "memory");
#if SB_LDS_BATCH > 0
            constexpr int BQ = SB_LDS_BATCH < RB ? SB_LDS_BATCH : RB;
#if SB_LDS_BATCH_ADDR
            // the rounds' topics first, so that every read below issues back
            // to back (no address arithmetic between them to reuse a register
            // still awaited)
            int tq[BQ];
#pragma unroll
            for (int q = 0; q < BQ; ++q) tq[q] = (int)(ring[s][q] & ENT_TOPIC_MASK);
            __builtin_amdgcn_sched_barrier(0);
#endif
            const DocReads dr = doc_reads();
            // every batched round's reads (a round past the row reads topic
            // 0's entries: harmless, its count is 0 and it is skipped below)
            float2 tbq[BQ];
            int ndq[BQ];
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
#if SB_LDS_BATCH_ADDR
              const int t_ = tq[q];
#else
              const int t_ = (int)(ring[s][q] & ENT_TOPIC_MASK);
#endif
              tbq[q] = tab[t_];
              ndq[q] = nd16_get(nd2, t_);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
              if (q < SB_RU || q < nr_all) {
                const float coef = __builtin_fmaf((float)ndq[q], tbq[q].x, tbq[q].y);
                acc = __builtin_fmaf((float)(ring[s][q] >> ENT_TOPIC_BITS), coef, acc);
              }
              accq[q] = acc;
            }
            doc_part(dr);
#if SB_LDS_BATCH2 > 0
            constexpr int BQ2 = (BQ + SB_LDS_BATCH2 < RB ? BQ + SB_LDS_BATCH2 : RB);
            if (BQ2 > BQ && nr_all > BQ) {
              float2 tb2[BQ2 > BQ ? BQ2 - BQ : 1];
              int nd2q[BQ2 > BQ ? BQ2 - BQ : 1];
#pragma unroll
              for (int q = BQ; q < BQ2; ++q) {
                const int t_ = (int)(ring[s][q] & ENT_TOPIC_MASK);
                tb2[q - BQ] = tab[t_];
                nd2q[q - BQ] = nd16_get(nd2, t_);
              }
              __builtin_amdgcn_sched_barrier(0);
#pragma unroll
              for (int q = BQ; q < BQ2; ++q) {
                if (q < nr_all) {
                  const float coef = __builtin_fmaf((float)nd2q[q - BQ], tb2[q - BQ].x, tb2[q - BQ].y);
                  acc = __builtin_fmaf((float)(ring[s][q] >> ENT_TOPIC_BITS), coef, acc);
                }
                accq[q] = acc;
              }
            } else {
#pragma unroll
              for (int q = BQ; q < BQ2; ++q) accq[q] = acc;
            }
            rounds(false, BQ2);
#else
            rounds(false, BQ);
#endif
#else
            const DocReads dr = doc_reads();
            // the doc reads issue first; nothing moves across (the scheduler
            // had issued them after the rounds' reads had been waited for)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < SB_RU; ++q) {
              acc = term_acc(ring[s][q], w, false, acc);
              accq[q] = acc;
            }
            doc_part(dr);
            rounds(false, SB_RU);
#endif
          } else {
            asm volatile("" ::: "memory");
            doc_part(doc_reads());
            rounds(true, 0);
          }
          // every register of this token's ring slot has landed on every path
          // (a row shorter than RB rounds skips the rest): otherwise the
          // compiler keeps them "in flight" across the loop and, when it
          // reuses them, waits for the NEXT token's prefetch (vmcnt counts
          // in order)
#pragma unroll
          for (int q = 0; q < RB; ++q) asm volatile("" ::"v"(ring[s][q]));

          float accb[SB_NB];
#pragma unroll
          for (int i = 0; i < SB_NB; ++i) accb[i] = 0.0f;
          // the rounds past RB (long rows), streamed in double-buffered batches
          auto batches = [&](bool sat) {
            const __amdgpu_buffer_rsrc_t rb =
                __builtin_amdgcn_make_buffer_rsrc((void*)erow, (short)0, n * 4, kBufWord3);
            uint32_t ea[SB_BATCH];
            int lo4 = lane * 4;
            asm volatile("" : "+v"(lo4));
#if SB_EARLY_BATCH
#pragma unroll
            for (int b = 0; b < SB_BATCH; ++b) ea[b] = ea0[b];
#else
#pragma unroll
            for (int b = 0; b < SB_BATCH; ++b)
              ea[b] = __builtin_amdgcn_raw_buffer_load_b32(rb, lo4 + (RB + b) * 256, 0, 0);
#endif
            int mb = 0;
            for (int q0 = RB; q0 < nr_all; q0 += SB_BATCH, ++mb) {
              // the next batch's loads only when it exists: a load left
              // unconsumed keeps its registers "in flight" into the next token
              uint32_t en[SB_BATCH];
#if SB_EARLY_BATCH >= 2
              if (q0 == RB) {
#pragma unroll
                for (int b = 0; b < SB_BATCH; ++b) en[b] = eb0[b];
              } else
#endif
              if (q0 + SB_BATCH < nr_all) {
                const int vo = lo4 + (q0 + SB_BATCH) * 256;
#pragma unroll
                for (int b = 0; b < SB_BATCH; ++b) en[b] = __builtin_amdgcn_raw_buffer_load_b32(rb, vo + b * 256, 0, 0);
              } else {
#pragma unroll
                for (int b = 0; b < SB_BATCH; ++b) en[b] = 0u;
              }
#if SB_LDS_BATCH_LONG
              if (!sat) {
                // the batch's LDS reads issued together (one round trip per
                // batch instead of one per round), then its fma in order
                float2 tbb[SB_BATCH];
                int ndb[SB_BATCH];
#pragma unroll
                for (int b = 0; b < SB_BATCH; ++b) {
                  const int t_ = (int)(ea[b] & ENT_TOPIC_MASK);
                  tbb[b] = tab[t_];
                  ndb[b] = nd16_get(nd2, t_);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int b = 0; b < SB_BATCH; ++b) {
                  const float coef = __builtin_fmaf((float)ndb[b], tbb[b].x, tbb[b].y);
                  acc = __builtin_fmaf((float)(ea[b] >> ENT_TOPIC_BITS), coef, acc);
                }
              } else {
#pragma unroll
                for (int b = 0; b < SB_BATCH; ++b) acc = term_acc(ea[b], w, sat, acc);
              }
#else
#pragma unroll
              for (int b = 0; b < SB_BATCH; ++b) acc = term_acc(ea[b], w, sat, acc);
#endif
#pragma unroll
              for (int i = 0; i < SB_NB; ++i) accb[i] = (mb == i) ? acc : accb[i];
#pragma unroll
              for (int b = 0; b < SB_BATCH; ++b) ea[b] = en[b];
            }
          };
          auto refill = [&]() {
            // every use of this token's ring slot is above: refill the slot
            // of token t-1 (the loads cannot move above this point)
            asm volatile("" : "+v"(acc)::"memory");
            const int sp = (s + NS - 1) % NS;
            prefetch(ring[sp], rm1[sp], t + NS - 1);
          };
#if SB_REFILL_LAST
          if (nr_all > RB) {
            if (!row_sat) batches(false);
            else batches(true);
          }
#else
#if !SB_REFILL_FIRST
          refill();
#else
          (void)refill;
#endif
          if (nr_all > RB) {
            if (!row_sat) batches(false);
            else batches(true);
          }
#endif
          const float TB = wave_incl_scan(acc);
          const float sumB = readlane_f(TB, 63);

          // the serial re-walk of lane lstar's rounds [r0, r1) from a0: the
          // first whose running sum exceeds thrE, else the last; its entry
          // and the running sums before / after it (the sums are those of the
          // rounds, fma for fma)
          struct Walk {
            uint32_t e;
            float lo, hi;
          };
          auto rewalk = [&](int lstar, int r0, int r1, float a, float thrE) -> Walk {
            const int nx = r1 - r0;
            const uint32_t ex = lane < nx ? erow[lstar + 64 * (r0 + lane)] : 0u;
            float cf, cof;
            term_parts(ex, w, row_sat, cf, cof);
            int sel = nx - 1;
            float lo = a, hi = a;
            for (int q = 0; q < nx; ++q) {
              lo = a;
              a = __builtin_fmaf(readlane_f(cf, q), readlane_f(cof, q), a);
              hi = a;
              if (a > thrE) {
                sel = q;
                break;
              }
            }
            return Walk{(uint32_t)readlane_i((int)ex, sel), lo, hi};
          };
          // A: tfx in fixed point; the alpha part (prefix of G'), then the
          // document part (prefix of nd F'), topics ascending
          auto pick_a = [&](float thr) -> int {
            const float t2 = thr - sumB;
            const uint64_t tfx = d2u64((double)t2 * isig);
            if (tfx < As) {
              SB_COUNT(1);
#if SB_APICK_LDS
              // the block of C topics: the block-end prefixes of G' (one
              // global read); within it the prefix from LDS: G' = fixp(ainv)
              // (+ dG at zo) split in 16-bit halves, each scanned in 32-bit
              // lanes (< 2^22), so no second global round trip
              const int kc = C * lane + C - 1;
#if SB_PFX_REG
              const uint64_t pc = pfx_r;
#else
              const uint64_t pc = KGLOBAL(big.pfx)[kc];
#endif
              const int64_t vc = (int64_t)pc + ((!FROZEN && kc >= zo) ? dG : 0);
              const uint64_t mc = __ballot((uint64_t)vc > tfx);
              const int L = mc ? (int)__builtin_ctzll(mc) : 63;
              const int kb = C * L - 1;    // the topic before the block
              const uint64_t pb = L > 0 ? (((uint64_t)(uint32_t)readlane_i((int)(uint32_t)(pc >> 32), L - 1) << 32) |
                                           (uint32_t)readlane_i((int)(uint32_t)pc, L - 1))
                                        : 0ull;
              const uint64_t El = pb + (uint64_t)((!FROZEN && L > 0 && kb >= zo) ? dG : 0);
              const int kf = C * L + lane;
              uint32_t g = 0;
              if (lane < C) g = fixp(tab[kf].y) + (uint32_t)((!FROZEN && kf == zo) ? dG : 0);
              const uint32_t slo = (uint32_t)wave_incl_scan_i((int)(g & 0xFFFFu));
              const uint32_t shi = (uint32_t)wave_incl_scan_i((int)(g >> 16));
              const uint64_t incl = El + ((uint64_t)shi << 16) + slo;
              const uint64_t mf = __ballot(lane < C && incl > tfx);
              const int k = mf ? C * L + (int)__builtin_ctzll(mf) : last_topic;
#else
              const int kc = C * lane + C - 1;
              const int64_t vc = (int64_t)KGLOBAL(big.pfx)[kc] + ((!FROZEN && kc >= zo) ? dG : 0);
              const uint64_t mc = __ballot((uint64_t)vc > tfx);
              const int L = mc ? (int)__builtin_ctzll(mc) : 63;
              const int kf = C * L + (lane < C ? lane : C - 1);
              const int64_t vf = (int64_t)KGLOBAL(big.pfx)[kf] + ((!FROZEN && kf >= zo) ? dG : 0);
              const uint64_t mf = __ballot(lane < C && (uint64_t)vf > tfx);
              const int k = mf ? C * L + (int)__builtin_ctzll(mf) : last_topic;
#endif
              return k < last_topic ? k : last_topic;
            }
            const uint64_t tr = tfx - As;
            SB_COUNT(2);
#if SB_APICK_LDS
            // lane l's topics [C l, C l + C), counts and F (= fixp(inv), as
            // k_big_tables makes it) from LDS, each lane starting its walk
            // at its own lane index: at the 2C-word lane stride of the
            // tables, lanes in step would hit one bank (round 5 had read F
            // from global memory, one round trip per 8 topics: the document
            // part of A was ~4% of the draws near init and most of their
            // time); the own topic's F' = Fm1 added as a correction on its lane
            uint64_t ps = 0;
            {
#if SB_ADOC_SPARSE && !SB_ND8
              // only the lane's nonzero count words: a mask from C / 8
              // 16-byte reads (starting at a lane-rotated chunk), then one
              // count word and one 16-byte tab read per nonzero word (a
              // document holds at most a few hundred topics of 4096); the
              // same integer sum, in another order
              const uint4* ndv = reinterpret_cast<const uint4*>(nd2) + lane * (C / 8);
              uint32_t nzm = 0;
#pragma unroll 2
              for (int j8 = 0; j8 < C / 8; ++j8) {
                const int o8 = (j8 + lane) & (C / 8 - 1);
                const uint4 v = ndv[o8];
                const uint32_t b = (uint32_t)(v.x != 0u) | ((uint32_t)(v.y != 0u) << 1) |
                                   ((uint32_t)(v.z != 0u) << 2) | ((uint32_t)(v.w != 0u) << 3);
                nzm |= b << (4 * o8);
              }
              const float2* tl = tab + C * lane;
              const uint32_t* ndw = nd2 + lane * (C / 2);
              // a wave-uniform loop (a lane out of words adds 0): a divergent
              // one made the allocator spill ~90 VGPRs
              while (__ballot(nzm != 0u)) {
                const bool has = nzm != 0u;
                const int i = has ? __builtin_ctz(nzm) : 0;
                nzm &= nzm - 1u;
                const uint32_t wv = has ? ndw[i] : 0u;
                const float4 t2 = *reinterpret_cast<const float4*>(tl + 2 * i);
                ps += (uint64_t)(wv & 0xFFFFu) * fixp(t2.x) + (uint64_t)(wv >> 16) * fixp(t2.z);
              }
#else
#if SB_ND8
              const uint8_t* ndh = reinterpret_cast<const uint8_t*>(nd2) + C * lane;
#else
              const uint16_t* ndh = reinterpret_cast<const uint16_t*>(nd2) + C * lane;
#endif
              const float2* tl = tab + C * lane;
#pragma unroll 8
              for (int j = 0; j < C; ++j) {
                const int o = (j + lane) & (C - 1);
                ps += (uint64_t)ndh[o] * fixp(tl[o].x);
              }
#endif
              if (!FROZEN && lane == (int)((uint32_t)zo / (uint32_t)C))
                ps += (uint64_t)((int64_t)ndz * ((int64_t)Fm1z - (int64_t)Fz));
            }
#else
            // lane l's topics [C l, C l + C): the counts as 16-byte LDS reads
            // (single u16 reads at a 2C-byte lane stride all hit one bank),
            // F as 16-byte global reads; the own topic's F' = Fm1 added as a
            // correction on its lane
            uint64_t ps = 0;
            {
              const uint4* ndv = reinterpret_cast<const uint4*>(nd2 + lane * (C / 2));
              const uint4* fv = reinterpret_cast<const uint4*>(KARG(big.F) + C * lane);
#pragma unroll 1
              for (int j8 = 0; j8 < C / 8; ++j8) {
                const uint4 nv = ndv[j8];
                const uint4 f0 = fv[2 * j8], f1 = fv[2 * j8 + 1];
                ps += (uint64_t)(nv.x & 0xFFFFu) * f0.x + (uint64_t)(nv.x >> 16) * f0.y;
                ps += (uint64_t)(nv.y & 0xFFFFu) * f0.z + (uint64_t)(nv.y >> 16) * f0.w;
                ps += (uint64_t)(nv.z & 0xFFFFu) * f1.x + (uint64_t)(nv.z >> 16) * f1.y;
                ps += (uint64_t)(nv.w & 0xFFFFu) * f1.z + (uint64_t)(nv.w >> 16) * f1.w;
              }
              if (!FROZEN && lane == (int)((uint32_t)zo / (uint32_t)C))
                ps += (uint64_t)((int64_t)ndz * ((int64_t)Fm1z - (int64_t)Fz));
            }
#endif
            const uint64_t incl = wave_incl_scan_u64(ps);
            const uint64_t ml = __ballot(incl > tr);
            if (!ml) return last_topic;
            const int L = (int)__builtin_ctzll(ml);
            const uint64_t El = L > 0 ? (((uint64_t)(uint32_t)readlane_i((int)(uint32_t)(incl >> 32), L - 1) << 32) |
                                          (uint32_t)readlane_i((int)(uint32_t)incl, L - 1))
                                       : 0ull;
            const int kf = C * L + (lane < C ? lane : C - 1);
#if SB_APICK_LDS
            const uint32_t ff = (!FROZEN && kf == zo) ? Fm1z : fixp(tab[kf].x);
#else
            const uint32_t ff = (!FROZEN && kf == zo) ? Fm1z : KGLOBAL(big.F)[kf];
#endif
            const uint64_t wf = lane < C ? (uint64_t)nd16_get(nd2, kf) * ff : 0ull;
            const uint64_t i2 = wave_incl_scan_u64(wf);
            const uint64_t mf = __ballot(lane < C && El + i2 > tr);
            const int k = mf ? C * L + (int)__builtin_ctzll(mf) : last_topic;
            return k < last_topic ? k : last_topic;
          };

          // the draw: B (lane, then round: register rounds, kept batch sums,
          // one re-walk), else A.  qsel >= 0: the entry is register round
          // qsel of lane lstar (its sums are read only for the own check)
          const float T = sumB + A_f;
          const float thr = uniform_f(u * T);
          SB_COUNT(0);
          int kn, lstar = -1, qsel = -1;
          Walk wk{0u, 0.0f, 0.0f};
          if (thr < sumB) {
            const int nl = n < 64 ? n : 64;
            const uint64_t m = __ballot((TB > thr) && (lane < nl));
            lstar = m ? (int)__builtin_ctzll(m) : nl - 1;
            const float E = lstar > 0 ? readlane_f(TB, lstar - 1) : 0.0f;
            const float thrE = thr - E;
            const int nr = (n - lstar + 63) >> 6;   // rounds of lane lstar
            int cv = 0;
#pragma unroll
            for (int q = 0; q < RB; ++q) cv += (accq[q] <= thrE) ? 1 : 0;
            const int cnt = readlane_i(cv, lstar);
            if (cnt < nr && cnt < RB) {
              qsel = cnt;
            } else if (nr <= RB) {
              qsel = nr - 1;
            } else {
              // lane lstar's rounds past RB: the first kept batch whose end
              // sum exceeds, else the rest; one re-walk of it
              const int nbl = (nr - RB + SB_BATCH - 1) / SB_BATCH;
              int cb = 0;
#pragma unroll
              for (int i = 0; i < SB_NB; ++i)
                if (i < nbl && cb == i && readlane_f(accb[i], lstar) <= thrE) cb = i + 1;
              int r0, r1;
              float a;
              if (cb < nbl && cb < SB_NB) {
                r0 = RB + SB_BATCH * cb;
                r1 = min(nr, r0 + SB_BATCH);
                a = readlane_f(accq[RB - 1], lstar);
#pragma unroll
                for (int i = 0; i < SB_NB; ++i)
                  if (cb == i + 1) a = readlane_f(accb[i], lstar);
              } else if (cb < nbl) {
                r0 = RB + SB_BATCH * SB_NB;
                r1 = nr;
                a = readlane_f(accb[SB_NB - 1], lstar);
              } else {
                // none exceeds: the lane's last batch (its last round is taken)
                r0 = RB + SB_BATCH * (nbl - 1);
                r1 = nr;
                a = readlane_f(accq[RB - 1], lstar);
#pragma unroll
                for (int i = 0; i < SB_NB; ++i)
                  if (nbl - 1 == i + 1) a = readlane_f(accb[i], lstar);
              }
              wk = rewalk(lstar, r0, r1, a, thrE);
            }
            if (qsel >= 0) wk.e = (uint32_t)readlane_i((int)ring[s][qsel], lstar);
            kn = (int)(wk.e & ENT_TOPIC_MASK);
          } else {
            kn = pick_a(thr);
          }
#ifdef SB_X_NOOWN
          if (false) {   // attribution experiment only (wrong draws)
#else
          if (!FROZEN && lstar >= 0 && kn == zo) {
#endif
            // the own entry: keep zo with probability O / w, else one re-draw
            // with the entry's width replaced by O
            SB_COUNT(3);
            if (qsel >= 0) {
              wk.hi = readlane_f(accq[qsel], lstar);
              wk.lo = qsel > 0 ? readlane_f(accq[qsel > 0 ? qsel - 1 : 0], lstar) : 0.0f;
            }
            uint32_t c = wk.e >> ENT_TOPIC_BITS;
            if (row_sat && c == ENT_COUNT_SAT) c = (uint32_t)KGLOBAL(nw)[(int64_t)w * KP + zo];
            const float wo = wk.hi - wk.lo;
            const float4 m1 = rm1[s];
            const float O = (float)(c > 0 ? c - 1 : 0u) * __builtin_fmaf((float)ndz, m1.x, m1.y);
#if SB_X1_LAZY
            // x1 of the token's Philox block computed here, on the own-entry
            // path only, instead of held per lane for the whole chunk
            uint32_t gt = (uint32_t)t;
            asm volatile("" : "+s"(gt));
            uint32_t y0, y1, y2;
            philox_x012(gbase + (uint64_t)gt, p.c2, p.c3, p.k0, p.k1, y0, y1, y2);
            const float u1 = u01(y1);
#else
            const float u1 = u01((uint32_t)readlane_i((int)cx1, idx));
#endif
            if (!(u1 * wo < O)) {
              // the re-draw (rare): x2 of the token's Philox block, computed
              // here (the token index passes an opaque register, so the block
              // is not hoisted into every token)
              SB_COUNT(4);
#if !SB_X1_LAZY
              uint32_t gt = (uint32_t)t;
              asm volatile("" : "+s"(gt));
              uint32_t y0, y1, y2;
              philox_x012(gbase + (uint64_t)gt, p.c2, p.c3, p.k0, p.k1, y0, y1, y2);
#endif
              const float s_lo = (lstar > 0 ? readlane_f(TB, lstar - 1) : 0.0f) + wk.lo;
              const float Tp = ((sumB - wo) + O) + A_f;
              const float thr2 = uniform_f(u01(y2) * Tp);
              if (!(thr2 >= s_lo && thr2 < s_lo + O)) {
                const float th = thr2 < s_lo ? thr2 : uniform_f((thr2 - O) + wo);
                // the same selection over the same sums, the lane's rounds
                // re-walked from memory (rows just read: in L2)
                if (th < sumB) {
                  const int nl = n < 64 ? n : 64;
                  const uint64_t m = __ballot((TB > th) && (lane < nl));
                  const int l2 = m ? (int)__builtin_ctzll(m) : nl - 1;
                  const float E = l2 > 0 ? readlane_f(TB, l2 - 1) : 0.0f;
                  const int nr = (n - l2 + 63) >> 6;
                  kn = (int)(rewalk(l2, 0, nr, 0.0f, th - E).e & ENT_TOPIC_MASK);
                } else {
                  kn = pick_a(th);
                }
              }
            }
          }
#if SB_REFILL_LAST
          // the refill after every load of this token (rare paths' waits
          // would otherwise drain it; the next token's waits still count it)
          refill();
#endif
          pk = kn;
          cn = (lane == idx) ? kn : cn;
#if SB_TOKEN_LGKM0
          // every LDS read of this token has been used by now: say so, so the
          // waitcnt pass does not carry a rare path's pending LDS write into
          // the next token's first reads as an lgkmcnt(0)
          __builtin_amdgcn_s_waitcnt(kLgkmcnt0);
#endif
        }
      }
    }
    flush_chunk();
    if (cbase + lane < t1) zr[cbase + lane] = cn;
    clear_doc();
  }
}


// Row capacities min(Kp, word total) (one wave per row).
__global__ __launch_bounds__(256) void k_row_caps(const int32_t* __restrict__ nw, int64_t V,
                                                  int32_t Kp, int32_t* __restrict__ caps) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * 4 + wid; w < V; w += (int64_t)gridDim.x * 4) {
    int64_t tot = 0;
    for (int k = lane; k < Kp; k += 64) tot += nw[w * Kp + k];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) tot += __shfl_xor(tot, o);
    if (lane == 0) caps[w] = (int32_t)(tot < Kp ? tot : Kp);
  }
}

// Compact every nw row into its sparse entries, topic ascending, zero-padded
// to a whole number of 64-entry rounds (one wave per row).
template <int C>
__global__ __launch_bounds__(256) void k_build_sparse(const int32_t* __restrict__ nw, int64_t V,
                                                      const int64_t* __restrict__ row_off,
                                                      uint32_t* __restrict__ ent,
                                                      int32_t* __restrict__ row_nnz) {
  constexpr int KP = C * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t w = (int64_t)blockIdx.x * 4 + wid; w < V; w += (int64_t)gridDim.x * 4) {
    int32_t c[C];
    load_row<C>(c, nw + w * KP + lane * C);
    int cnt = 0;
    bool sat = false;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      cnt += c[j] > 0 ? 1 : 0;
      sat |= (uint32_t)c[j] >= ENT_COUNT_SAT;
    }
    const bool row_sat = __ballot(sat) != 0;
    const int incl = wave_incl_scan_i(cnt);
    int pos = incl - cnt;
    const int64_t o = row_off[w];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (c[j] > 0) {
        const uint32_t cc = (uint32_t)c[j] >= ENT_COUNT_SAT ? ENT_COUNT_SAT : (uint32_t)c[j];
        ent[o + pos] = (cc << ENT_TOPIC_BITS) | (uint32_t)(lane * C + j);
        ++pos;
      }
    }
    // zero entries up to the next whole round of 64 (the capacity is padded
    // to whole rounds): the large-K sampler loads full rounds, and a zero
    // entry adds +0 to its sums
    const int nnz = __shfl(incl, 63);
    const int pad_end = (nnz + 63) & ~63;
    if (nnz + lane < pad_end) ent[o + nnz + lane] = 0u;
    // sign bit: the row holds a saturated count (the sampler then checks
    // entries for the escape; otherwise it skips that per-entry branch)
    if (lane == 63) row_nnz[w] = row_sat ? (int32_t)((uint32_t)incl | 0x80000000u) : incl;
  }
}

// the draws of given global token indices (lda_philox_draws diagnostics)
__global__ __launch_bounds__(256) void k_philox_draws(const int64_t* __restrict__ gtok, int64_t n,
                                                      uint32_t c2, uint32_t c3, uint32_t k0,
                                                      uint32_t k1, uint32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    out[i] = draw_u32((uint64_t)gtok[i], c2, c3, k0, k1);
}

// ----------------------------------------------------------- count kernels
__global__ __launch_bounds__(256) void k_init_z(int32_t* __restrict__ z, int64_t n, int32_t K,
                                                int64_t token_base, uint32_t k0, uint32_t k1) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t x = draw_u32((uint64_t)(token_base + i), 0u, STREAM_INIT, k0, k1);
    z[i] = (int32_t)(((uint64_t)x * (uint64_t)K) >> 32);
  }
}

// Local histogram of (word, topic) and topic totals into the delta buffer.
__global__ __launch_bounds__(256) void k_count(const int32_t* __restrict__ words,
                                               const int32_t* __restrict__ z, int64_t n,
                                               int32_t Kp, int32_t* __restrict__ delta,
                                               int32_t* __restrict__ dsum) {
  extern __shared__ __attribute__((aligned(16))) int32_t hsum[];
  for (int i = threadIdx.x; i < Kp; i += 256) hsum[i] = 0;
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int k = z[i];
    atomicAdd(&delta[(int64_t)words[i] * Kp + k], 1);
    atomicAdd(&hsum[k], 1);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < Kp; i += 256)
    if (hsum[i]) atomicAdd(&dsum[i], hsum[i]);
}

// nw += delta; delta = 0 over the V*Kp region (Kp is a multiple of 64, so
// the region is a multiple of 4 int32 and int4-aligned).
__global__ __launch_bounds__(256) void k_apply(int4* __restrict__ nw, int4* __restrict__ delta,
                                               int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    int4 a = nw[i];
    const int4 d = delta[i];
    if (d.x | d.y | d.z | d.w) {
      a.x += d.x;
      a.y += d.y;
      a.z += d.z;
      a.w += d.w;
      nw[i] = a;
      delta[i] = make_int4(0, 0, 0, 0);
    }
  }
}

// The sparse samplers' apply: nw += delta; delta = 0 over the V*Kp cells
// (int4 groups that are zero in delta are not rewritten), and dsum += the
// column sums of the delta -- the nwsum delta, which the sparse samplers do
// not write (their per-token nwsum atomics all hit one Kp-cell array).  The
// grid is a multiple of kp4 = Kp/4 threads, so thread t owns int4 column
// group t % kp4 of every row it visits and keeps its partial sums in four
// registers: one device atomic per nonzero partial at the end (~Kp per 256
// blocks) instead of two per changed token.
__global__ __launch_bounds__(256) void k_apply_cols(int4* __restrict__ nw, int4* __restrict__ delta,
                                                    int64_t n4, int32_t* __restrict__ dsum, int32_t kp4) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t T = (int64_t)gridDim.x * 256;
  int4 acc = make_int4(0, 0, 0, 0);
  for (int64_t i = gid; i < n4; i += T) {
    const int4 d = delta[i];
    if (d.x | d.y | d.z | d.w) {
      int4 a = nw[i];
      a.x += d.x;
      a.y += d.y;
      a.z += d.z;
      a.w += d.w;
      nw[i] = a;
      delta[i] = make_int4(0, 0, 0, 0);
      acc.x += d.x;
      acc.y += d.y;
      acc.z += d.z;
      acc.w += d.w;
    }
  }
  int32_t* ds = dsum + (gid % kp4) * 4;
  if (acc.x) atomicAdd(ds + 0, acc.x);
  if (acc.y) atomicAdd(ds + 1, acc.y);
  if (acc.z) atomicAdd(ds + 2, acc.z);
  if (acc.w) atomicAdd(ds + 3, acc.w);
}

// The sparse samplers' apply fused with the row build (round 4): one wave per
// word row reads its nw and delta rows once, writes nw += delta and delta = 0
// for the int4 groups that changed, accumulates the column sums of the delta
// (the nwsum delta) in lane-private LDS words, and builds the row's sparse
// entries from the updated counts still in registers -- k_apply_cols +
// k_build_sparse without the second full read of nw.  Lane l owns topics
// [l*C, l*C+C), as k_build_sparse.  At the end the block's waves add their
// column sums and one atomic per nonzero column goes to dsum.
template <int C>
__global__ __launch_bounds__(256) void k_apply_build(int32_t* __restrict__ nw, int32_t* __restrict__ delta,
                                                     int64_t V, const int64_t* __restrict__ row_off,
                                                     uint32_t* __restrict__ ent, int32_t* __restrict__ row_nnz,
                                                     int32_t* __restrict__ dsum) {
  constexpr int KP = C * 64;
  extern __shared__ __attribute__((aligned(16))) int32_t smem[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t* cs = smem + wid * KP + lane * C;          // this lane's column sums
#pragma unroll
  for (int j = 0; j < C; ++j) cs[j] = 0;
  for (int64_t w = (int64_t)blockIdx.x * 4 + wid; w < V; w += (int64_t)gridDim.x * 4) {
    int32_t c[C], d[C];
    int32_t* nrow = nw + w * KP + lane * C;
    int32_t* drow = delta + w * KP + lane * C;
    load_row<C>(c, nrow);
    load_row<C>(d, drow);
#pragma unroll
    for (int q = 0; q < (C + 3) / 4; ++q) {
      const int n = C < 4 ? C : 4;
      bool ch = false;
#pragma unroll
      for (int i = 0; i < n; ++i) ch |= d[4 * q + i] != 0;
      if (ch) {
#pragma unroll
        for (int i = 0; i < n; ++i) {
          c[4 * q + i] += d[4 * q + i];
          nrow[4 * q + i] = c[4 * q + i];
          drow[4 * q + i] = 0;
          cs[4 * q + i] += d[4 * q + i];
        }
      }
    }
    int cnt = 0;
    bool sat = false;
#pragma unroll
    for (int j = 0; j < C; ++j) {
      cnt += c[j] > 0 ? 1 : 0;
      sat |= (uint32_t)c[j] >= ENT_COUNT_SAT;
    }
    const bool row_sat = __ballot(sat) != 0;
    const int incl = wave_incl_scan_i(cnt);
    int pos = incl - cnt;
    const int64_t o = row_off[w];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      if (c[j] > 0) {
        const uint32_t cc = (uint32_t)c[j] >= ENT_COUNT_SAT ? ENT_COUNT_SAT : (uint32_t)c[j];
        ent[o + pos] = (cc << ENT_TOPIC_BITS) | (uint32_t)(lane * C + j);
        ++pos;
      }
    }
    const int nnz = __shfl(incl, 63);
    const int pad_end = (nnz + 63) & ~63;
    if (nnz + lane < pad_end) ent[o + nnz + lane] = 0u;
    if (lane == 63) row_nnz[w] = row_sat ? (int32_t)((uint32_t)incl | 0x80000000u) : incl;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KP; i += 256) {
    const int v = smem[i] + smem[KP + i] + smem[2 * KP + i] + smem[3 * KP + i];
    if (v != 0) atomicAdd(&dsum[i], v);
  }
}

// ---- compact exchange (lda_exchange_pack / lda_exchange_unpack)
// Two exchange cells per int32 word, biased so that the SUM over `world`
// ranks cannot carry between the halves: cell 2i as d + b0 in bits 0..15
// (b0 = 2^15 / world, so the sum stays below 2^16), cell 2i+1 as d + b1 in
// bits 16..30 (b1 = 2^14 / world: the word's sum stays below 2^31, no int32
// overflow in the collective).  A cell outside [-b, b) packs as b (a zero
// change) and goes to the escape list {count, (cell lo, cell hi, value)...}
// instead; every rank's list is all-gathered and added after the unpack.
// Sum |d| over a shard's cells is at most 2 x its tokens (each changed token
// is -1 and +1; a recount buffer holds counts summing to the tokens), so at
// most 2 N / b1 cells can escape: the caller's capacity (lda_exchange_sizes).
__device__ __forceinline__ uint32_t exch_field(int32_t d, int32_t b, int64_t cell, int32_t* __restrict__ esc,
                                               int32_t cap) {
  if (d >= -b && d < b) return (uint32_t)(d + b);
  const int pos = atomicAdd(esc, 1);
  if (pos < cap) {
    int32_t* e = esc + 1 + 3 * (int64_t)pos;
    e[0] = (int32_t)(uint32_t)cell;
    e[1] = (int32_t)(cell >> 32);
    e[2] = d;
  }
  return (uint32_t)b;
}

__global__ __launch_bounds__(256) void k_exch_pack(const int4* __restrict__ buf, int64_t n4,
                                                   uint2* __restrict__ packed, int32_t b0, int32_t b1,
                                                   int32_t* __restrict__ esc, int32_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int4 d = buf[i];
    const int64_t c = 4 * i;
    const uint32_t w0 = exch_field(d.x, b0, c, esc, cap) | (exch_field(d.y, b1, c + 1, esc, cap) << 16);
    const uint32_t w1 = exch_field(d.z, b0, c + 2, esc, cap) | (exch_field(d.w, b1, c + 3, esc, cap) << 16);
    packed[i] = make_uint2(w0, w1);
  }
}

// four cells per word (lda_set_exchange_cells 4): cells 0..2 of an int4 in
// bytes 0..2 biased by b, cell 3 in bits 24..30 biased by bt (the sum over
// `world` ranks of values below 2 b stays below 2^8 in each low byte and below
// 2^7 in the top one: no carry between cells, no int32 overflow)
__global__ __launch_bounds__(256) void k_exch_pack4(const int4* __restrict__ buf, int64_t n4,
                                                    uint32_t* __restrict__ packed, int32_t b, int32_t bt,
                                                    int32_t* __restrict__ esc, int32_t cap) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int4 d = buf[i];
    const int64_t c = 4 * i;
    packed[i] = exch_field(d.x, b, c, esc, cap) | (exch_field(d.y, b, c + 1, esc, cap) << 8) |
                (exch_field(d.z, b, c + 2, esc, cap) << 16) | (exch_field(d.w, bt, c + 3, esc, cap) << 24);
  }
}
__global__ __launch_bounds__(256) void k_exch_unpack4(const uint32_t* __restrict__ packed, int64_t n4,
                                                      int4* __restrict__ buf, int32_t wb, int32_t wbt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const uint32_t p = packed[i];
    buf[i] = make_int4((int32_t)(p & 0xFFu) - wb, (int32_t)((p >> 8) & 0xFFu) - wb,
                       (int32_t)((p >> 16) & 0xFFu) - wb, (int32_t)(p >> 24) - wbt);
  }
}

// the summed words back into int32 cells (every cell written: the buffer
// held this rank's own changes before the exchange)
__global__ __launch_bounds__(256) void k_exch_unpack(const uint2* __restrict__ packed, int64_t n4,
                                                     int4* __restrict__ buf, int32_t wb0, int32_t wb1) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const uint2 p = packed[i];
    buf[i] = make_int4((int32_t)(p.x & 0xFFFFu) - wb0, (int32_t)(p.x >> 16) - wb1,
                       (int32_t)(p.y & 0xFFFFu) - wb0, (int32_t)(p.y >> 16) - wb1);
  }
}

// every rank's escapes (the all-gathered lists, `world` x (1 + 3 cap) int32)
// added into the cells; blocks [4r, 4r + 4) take rank r's list
__global__ __launch_bounds__(256) void k_exch_escapes(const int32_t* __restrict__ esc_all, int32_t cap,
                                                      int32_t* __restrict__ buf) {
  const int r = blockIdx.x >> 2;
  const int32_t* e = esc_all + (int64_t)r * (1 + 3 * (int64_t)cap);
  const int n = min(e[0], cap);
  for (int j = (blockIdx.x & 3) * 256 + threadIdx.x; j < n; j += 1024) {
    const int32_t* x = e + 1 + 3 * (int64_t)j;
    const int64_t cell = (int64_t)(uint32_t)x[0] | ((int64_t)x[1] << 32);
    atomicAdd(buf + cell, x[2]);
  }
}

// lda_counts_checksum: sum (mod 2^64) over the nonzero cells of nw and nwsum
// of mix64(index << 32 | value), index = w K + k for nw[w][k], V K + k for
// nwsum[k] (the Kp padding is skipped, so the hash is that of the V x K
// arrays lda_get_counts returns; oracle.counts_checksum).  One partial per
// block, summed on the host: a sum is order-free, so every replica of the
// same counts gives the same value whatever the launch geometry.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xBF58476D1CE4E5B9ull;
  x ^= x >> 27;
  x *= 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__device__ __forceinline__ uint64_t cell_hash(int64_t index, int32_t v) {
  return v ? mix64(((uint64_t)index << 32) | (uint32_t)v) : 0ull;
}

__global__ __launch_bounds__(256) void k_counts_checksum(const int4* __restrict__ nw, int64_t n4,
                                                         const int32_t* __restrict__ nwsum, int32_t K, int32_t Kp,
                                                         int64_t V, uint64_t* __restrict__ partial) {
  __shared__ uint64_t red[256];
  uint64_t s = 0;
  const int64_t q = Kp / 4;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int4 d = nw[i];
    const int64_t w = i / q;
    const int32_t k = (int32_t)(i - w * q) * 4;
    const int64_t base = w * K + k;
    if (k + 0 < K) s += cell_hash(base + 0, d.x);
    if (k + 1 < K) s += cell_hash(base + 1, d.y);
    if (k + 2 < K) s += cell_hash(base + 2, d.z);
    if (k + 3 < K) s += cell_hash(base + 3, d.w);
  }
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k < K; k += 256) s += cell_hash(V * K + k, nwsum[k]);
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

// Split sweep (lda_set_exchange_parts): dst += src; src = 0 over the whole
// [V*Kp | Kp] delta region (a multiple of 4 int32: Kp is a multiple of 64).
// int4 groups that are zero in src are neither written nor re-zeroed.
__global__ __launch_bounds__(256) void k_fold_delta(int4* __restrict__ dst, int4* __restrict__ src,
                                                    int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const int4 d = src[i];
    if (d.x | d.y | d.z | d.w) {
      int4 a = dst[i];
      a.x += d.x;
      a.y += d.y;
      a.z += d.z;
      a.w += d.w;
      dst[i] = a;
      src[i] = make_int4(0, 0, 0, 0);
    }
  }
}

// One pass per sweep for the dense sampler: nw += delta (rows with an
// all-zero delta are not rewritten), delta = 0, the 16-bit copy and wide
// flag of every row, and — in the first block — nwsum += dsum and the
// per-topic fp32 tables, plus the work-queue reset of the next lda_sample.
// Replaces k_apply + k_build_packed + k_prepare_topics (+ a memset): one
// read of nw instead of two and one launch instead of four.
template <int C>
__global__ __launch_bounds__(256) void k_apply_packed(int32_t* __restrict__ nw, int32_t* __restrict__ delta,
                                                      int64_t V, uint16_t* __restrict__ nw16,
                                                      uint8_t* __restrict__ wide, TopicTables t) {
  constexpr int KP = C * 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (blockIdx.x == 0) {
    int32_t* dsum = delta + V * KP;
    for (int k = threadIdx.x; k < KP; k += 256) {
      const int32_t s = t.absolute ? dsum[k] : t.nwsum[k] + dsum[k];
      t.nwsum[k] = s;
      dsum[k] = 0;
      if (k < t.K) {
        const float vb = t.state_dev ? __uint_as_float(t.state_dev[2]) : t.vbeta;
        t.alpha_f[k] = (float)t.alpha[k];
        t.inv[k] = 1.0f / ((float)s + vb);
        t.inv_m1[k] = 1.0f / ((float)(s - 1) + vb);
      } else {
        t.alpha_f[k] = 0.0f;
        t.inv[k] = 0.0f;
        t.inv_m1[k] = 0.0f;
      }
    }
    if (threadIdx.x == 0 && t.queue) *t.queue = 0;
    if (threadIdx.x == 0 && t.state_dev && t.advance) t.state_dev[0] += 1u;   // the next graph sweep's counter
  }
  for (int64_t w = (int64_t)blockIdx.x * 4 + wid; w < V; w += (int64_t)gridDim.x * 4) {
    int32_t c[C], d[C];
    load_row<C>(d, delta + w * KP + lane * C);
    if (t.absolute) {
      // the buffer holds the recounted counts (k_recount, summed across
      // shards): they replace the row, and the buffer is left zero
#pragma unroll
      for (int j = 0; j < C; ++j) {
        c[j] = d[j];
        nw[w * KP + lane * C + j] = c[j];
      }
    } else {
      load_row<C>(c, nw + w * KP + lane * C);
    }
    bool changed = false;
#pragma unroll
    for (int j = 0; j < C; ++j) changed |= d[j] != 0;
    if (changed) {
#pragma unroll
      for (int j = 0; j < C; ++j) {
        if (!t.absolute) {
          c[j] += d[j];
          nw[w * KP + lane * C + j] = c[j];
        }
        delta[w * KP + lane * C + j] = 0;
      }
    }
    bool big = false;
#pragma unroll
    for (int j = 0; j < C; ++j) big |= (uint32_t)c[j] > 0xFFFFu;
    // a wide word's whole 16-bit row is 0xFFFF: the quarter kernel reads its
    // "take the int32 row" flag from the row itself (k_sample_quarter)
    const uint64_t any = __ballot(big);
#pragma unroll
    for (int j = 0; j < C; ++j)
      nw16[w * KP + lane * C + j] = any ? (uint16_t)0xFFFFu : (uint16_t)c[j];
    if (lane == 0) wide[w] = any ? 1 : 0;
  }
}

// nwsum += dsum; dsum = 0; per-topic fp32 tables (one block, Kp <= 1024).
__global__ void k_prepare_topics(int32_t* __restrict__ nwsum, int32_t* __restrict__ dsum,
                                 const double* __restrict__ alpha, double beta, double vbeta,
                                 int32_t K, int32_t Kp, float* __restrict__ alpha_f,
                                 float* __restrict__ inv, float* __restrict__ inv_m1) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= Kp) return;
  const int32_t s = nwsum[k] + dsum[k];
  nwsum[k] = s;
  dsum[k] = 0;
  const float vb = (float)vbeta;
  if (k < K) {
    alpha_f[k] = (float)alpha[k];
    inv[k] = 1.0f / ((float)s + vb);
    inv_m1[k] = 1.0f / ((float)(s - 1) + vb);
  } else {
    alpha_f[k] = 0.0f;
    inv[k] = 0.0f;
    inv_m1[k] = 0.0f;
  }
  (void)beta;
}

// Dense nd rows: one wavefront per document.
__global__ __launch_bounds__(256) void k_doc_topics(const int32_t* __restrict__ z,
                                                    const int64_t* __restrict__ doc_off, int64_t D,
                                                    int32_t K, int32_t Kp, int32_t* __restrict__ out,
                                                    int accumulate) {
  extern __shared__ __attribute__((aligned(16))) int32_t h[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t* hist = h + wid * Kp;
  for (int i = lane; i < Kp; i += 64) hist[i] = 0;
  for (int64_t d = (int64_t)blockIdx.x * 4 + wid; d < D; d += (int64_t)gridDim.x * 4) {
    for (int64_t i = doc_off[d] + lane; i < doc_off[d + 1]; i += 64) atomicAdd(&hist[z[i]], 1);
    wave_lds_fence();
    for (int k = lane; k < K; k += 64) {
      const int32_t c = hist[k];
      if (accumulate)
        out[d * K + k] += c;
      else
        out[d * K + k] = c;
    }
    for (int k = lane; k < Kp; k += 64) hist[k] = 0;
    wave_lds_fence();
  }
}

// Mallet's Dirichlet.logGammaStirling in fp64.
__device__ double log_gamma_stirling(double z) {
  const double HALF_LOG_TWO_PI = 0.91893853320467274178;
  int shift = 0;
  while (z < 2) {
    z += 1.0;
    ++shift;
  }
  double result = HALF_LOG_TWO_PI + (z - 0.5) * log(z) - z + 1 / (12 * z) -
                  1 / (360 * z * z * z) + 1 / (1260 * z * z * z * z * z);
  while (shift > 0) {
    --shift;
    z -= 1.0;
    result -= log(z);
  }
  return result;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Document part of modelLogLikelihood: one wave per doc, per-block partials.
// The document's topic counts are built in LDS, then read back through the
// document's own tokens -- the first lane to take topic k (an LDS exchange
// with 0) adds its term -- so a document costs O(its tokens), not O(Kp)
// (C5, Kp = 4096, 200-token documents: a 20x smaller walk).  The fp64 sum
// order differs from the oracle's topic order; the bar is 1e-9 relative.
__global__ __launch_bounds__(256) void k_ll_docs(const int32_t* __restrict__ z,
                                                 const int64_t* __restrict__ doc_off, int64_t D,
                                                 const double* __restrict__ alpha, double alpha_sum,
                                                 int32_t K, int32_t Kp, double* __restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) int32_t h[];
  __shared__ double wsum[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t* hist = h + wid * Kp;
  for (int i = lane; i < Kp; i += 64) hist[i] = 0;
  wave_lds_fence();
  double acc = 0.0;
  for (int64_t d = (int64_t)blockIdx.x * 4 + wid; d < D; d += (int64_t)gridDim.x * 4) {
    const int64_t t0 = doc_off[d], t1 = doc_off[d + 1];
    for (int64_t i = t0 + lane; i < t1; i += 64) atomicAdd(&hist[z[i]], 1);
    wave_lds_fence();
    // every topic of the document is taken by exactly one lane, which also
    // leaves its cell zero for the next document
    for (int64_t i = t0 + lane; i < t1; i += 64) {
      const int k = z[i];
      const int32_t c = atomicExch(&hist[k], 0);
      if (c > 0) acc += log_gamma_stirling(alpha[k] + c) - log_gamma_stirling(alpha[k]);
    }
    if (lane == 0) acc -= log_gamma_stirling(alpha_sum + (double)(t1 - t0));
    wave_lds_fence();
  }
  (void)K;
  acc = wave_sum_d(acc);
  if (lane == 0) wsum[wid] = acc;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
}

// Word part: sum over nonzero nw cells of logGammaStirling(beta + count).
__global__ __launch_bounds__(256) void k_ll_words(const int32_t* __restrict__ nw, int64_t V,
                                                  int32_t K, int32_t Kp, double beta,
                                                  double* __restrict__ partial,
                                                  unsigned long long* __restrict__ nonzero) {
  __shared__ double wsum[4];
  __shared__ unsigned long long wnz[4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  double acc = 0.0;
  unsigned long long nz = 0;
  const int64_t n = V * Kp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int k = (int)(i % Kp);
    const int32_t c = nw[i];
    if (k < K && c > 0) {
      acc += log_gamma_stirling(beta + c);
      ++nz;
    }
  }
  acc = wave_sum_d(acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) nz += __shfl_xor(nz, o);
  if (lane == 0) {
    wsum[wid] = acc;
    wnz[wid] = nz;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partial[blockIdx.x] = ((wsum[0] + wsum[1]) + wsum[2]) + wsum[3];
    nonzero[blockIdx.x] = wnz[0] + wnz[1] + wnz[2] + wnz[3];
  }
}

// TopicInferencer init: most frequent topic of the word (ties -> larger id).
// Mallet's alpha statistics (WorkerRunnable, shouldSaveState): per document
// docLengthCounts[len]++ and topicDocCounts[k][n_dk]++ for every n_dk > 0;
// one wavefront per document, the document's counts in LDS.
// The block's counts of document lengths up to DOC_HIST_LEN and of (topic,
// count) pairs with count <= DOC_HIST_SMALL are summed in LDS and added to the
// device histograms once per block: the same few cells (common lengths, a
// topic held once) took every document's device atomic and serialised on it
// (25 us a launch at the reference's 2000 documents).
#define DOC_HIST_LEN 1024
#define DOC_HIST_SMALL 4
__global__ __launch_bounds__(256) void k_doc_hist(const int32_t* __restrict__ z,
                                                  const int64_t* __restrict__ doc_off, int64_t D,
                                                  int32_t K, int32_t Kp, int32_t L,
                                                  int32_t* __restrict__ len_hist,
                                                  int32_t* __restrict__ topic_hist) {
  extern __shared__ __attribute__((aligned(16))) int32_t h[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t* hist = h + wid * Kp;
  int32_t* len_l = h + 4 * Kp;                       // [DOC_HIST_LEN]
  int32_t* small = len_l + DOC_HIST_LEN;              // [K][DOC_HIST_SMALL], count c at c - 1
  for (int i = threadIdx.x; i < 4 * Kp + DOC_HIST_LEN + K * DOC_HIST_SMALL; i += 256) h[i] = 0;
  __syncthreads();
  for (int64_t d = (int64_t)blockIdx.x * 4 + wid; d < D; d += (int64_t)gridDim.x * 4) {
    const int64_t t0 = doc_off[d], t1 = doc_off[d + 1];
    for (int64_t i = t0 + lane; i < t1; i += 64) atomicAdd(&hist[z[i]], 1);
    wave_lds_fence();
    if (lane == 0) {
      const int64_t n = t1 - t0;
      if (n < DOC_HIST_LEN) atomicAdd(&len_l[n], 1);
      else atomicAdd(&len_hist[n], 1);
    }
    // each of the document's topics taken once through its tokens (as k_ll_docs)
    for (int64_t i = t0 + lane; i < t1; i += 64) {
      const int k = z[i];
      const int32_t c = atomicExch(&hist[k], 0);
      if (c > 0 && c <= DOC_HIST_SMALL) atomicAdd(&small[k * DOC_HIST_SMALL + c - 1], 1);
      else if (c > 0) atomicAdd(&topic_hist[(int64_t)k * (L + 1) + c], 1);
    }
    wave_lds_fence();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < DOC_HIST_LEN && i <= L; i += 256)
    if (len_l[i]) atomicAdd(&len_hist[i], len_l[i]);
  for (int i = threadIdx.x; i < K * DOC_HIST_SMALL; i += 256) {
    const int c = i % DOC_HIST_SMALL + 1;
    if (small[i] && c <= L) atomicAdd(&topic_hist[(int64_t)(i / DOC_HIST_SMALL) * (L + 1) + c], small[i]);
  }
}

// optimizeBeta's countHistogram: cells of nw (k < K) holding each count > 0.
// Small counts are binned in LDS first (they are most of the cells).
#define COUNT_HIST_LDS 4096
__global__ __launch_bounds__(256) void k_count_hist(const int32_t* __restrict__ nw, int64_t V,
                                                    int32_t K, int32_t Kp, int64_t max_count,
                                                    int32_t* __restrict__ hist,
                                                    int32_t* __restrict__ overflow) {
  __shared__ int32_t sh[COUNT_HIST_LDS];
  for (int i = threadIdx.x; i < COUNT_HIST_LDS; i += 256) sh[i] = 0;
  __syncthreads();
  const int64_t n = V * Kp;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int k = (int)(i & (Kp - 1));
    const int32_t c = nw[i];
    if (k < K && c > 0) {
      if ((int64_t)c > max_count)
        atomicOr(overflow, 1);
      else if (c < COUNT_HIST_LDS)
        atomicAdd(&sh[c], 1);
      else
        atomicAdd(&hist[c], 1);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < COUNT_HIST_LDS && i <= max_count; i += 256)
    if (sh[i]) atomicAdd(&hist[i], sh[i]);
}

// Token-weighted row sparsity of the snapshot: sum_w total_w * nnz_w and
// sum_w total_w (one wave per row, one pair of atomics per block).
__global__ __launch_bounds__(256) void k_row_stats(const int32_t* __restrict__ nw, int64_t V,
                                                   int32_t K, int32_t Kp,
                                                   unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[2][4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned long long wsum = 0, wtot = 0;
  for (int64_t w = (int64_t)blockIdx.x * 4 + wid; w < V; w += (int64_t)gridDim.x * 4) {
    unsigned long long tot = 0, nnz = 0;
    for (int k = lane; k < K; k += 64) {
      const int32_t c = nw[w * Kp + k];
      tot += (unsigned long long)c;
      nnz += c > 0 ? 1 : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      tot += __shfl_xor(tot, o);
      nnz += __shfl_xor(nnz, o);
    }
    wsum += tot * nnz;
    wtot += tot;
  }
  if (lane == 0) {
    part[0][wid] = wsum;
    part[1][wid] = wtot;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&out[0], part[0][0] + part[0][1] + part[0][2] + part[0][3]);
    atomicAdd(&out[1], part[1][0] + part[1][1] + part[1][2] + part[1][3]);
  }
}

__global__ __launch_bounds__(256) void k_infer_init(const int32_t* __restrict__ words,
                                                    int32_t* __restrict__ z, int64_t n,
                                                    const int32_t* __restrict__ nw, int32_t K,
                                                    int32_t Kp) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int64_t i = (int64_t)blockIdx.x * 4 + wid; i < n; i += (int64_t)gridDim.x * 4) {
    const int32_t* row = nw + (int64_t)words[i] * Kp;
    int best_c = -1, best_k = 0;
    for (int k = lane; k < K; k += 64) {
      const int c = row[k];
      if (c >= best_c) {
        best_c = c;
        best_k = k;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const int oc = __shfl_xor(best_c, o), ok = __shfl_xor(best_k, o);
      if (oc > best_c || (oc == best_c && ok > best_k)) {
        best_c = oc;
        best_k = ok;
      }
    }
    if (lane == 0) z[i] = best_k;
  }
}

// ---------------------------------------------------------------- recount
// The dense samplers' count update without atomics in the sampler (DESIGN
// §4 "Recount"): the sampler only writes z; afterwards every word's row of
// THIS shard is recounted from a word-sorted token index, and the result is
// the exchange buffer (summed across shards as Mallet's sumTypeTopicCounts
// sums its workers' local typeTopicCounts [M]); k_apply_packed then replaces
// nw by it.  Integer counts: the result does not depend on any order.

// tokens per (part, word): cnt[part * V + w]
__global__ __launch_bounds__(256) void k_word_hist(const int32_t* __restrict__ words, int64_t n,
                                                   PartSpans ps, int64_t V,
                                                   uint32_t* __restrict__ cnt) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int part = 0;
    while (part + 1 < ps.parts && i >= ps.tok[part + 1]) ++part;
    atomicAdd(&cnt[(int64_t)part * V + words[i]], 1u);
  }
}

// perm[cursor[part * V + w]++] = i: token indices grouped by (part, word)
// (the order inside a group is whatever the atomics give; nothing depends
// on it)
__global__ __launch_bounds__(256) void k_word_scatter(const int32_t* __restrict__ words, int64_t n,
                                                      PartSpans ps, int64_t V,
                                                      uint32_t* __restrict__ cursor,
                                                      uint32_t* __restrict__ perm) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int part = 0;
    while (part + 1 < ps.parts && i >= ps.tok[part + 1]) ++part;
    const uint32_t pos = atomicAdd(&cursor[(int64_t)part * V + words[i]], 1u);
    perm[pos] = (uint32_t)i;
  }
}

// One wave per work item {word, first perm index, tokens, split}: the
// item's topics are histogrammed in LDS (z gathered through perm, four
// 64-token loads in flight per lane), then the row goes out -- stored whole
// when the word is one item, added cell by cell (device atomics on the
// nonzero cells) when it is split over several; the buffer is zero on entry
// (k_apply_packed leaves it so).  The block's column sums go to bufsum.
// Items are dealt to waves round-robin (they are sorted longest first): a
// work-queue counter, one same-address atomic per item, had capped the
// kernel at ~60M items/s (C2: 0.81 ms for 50k items).
template <int C>
__global__ __launch_bounds__(256) void k_recount(const uint32_t* __restrict__ perm,
                                                 const int32_t* __restrict__ zw,
                                                 const int4* __restrict__ items, int32_t n_items,
                                                 const int32_t* __restrict__ z,
                                                 int32_t* __restrict__ buf,
                                                 int32_t* __restrict__ bufsum) {
  constexpr int KP = C * 64;
  __shared__ __attribute__((aligned(16))) int32_t lds[5 * KP];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int32_t* hist = lds + wid * KP;
  int32_t* bs = lds + 4 * KP;
  for (int i = threadIdx.x; i < 5 * KP; i += 256) lds[i] = 0;
  __syncthreads();
  for (int it = (int)blockIdx.x * 4 + wid; it < n_items; it += (int)gridDim.x * 4) {
    const int4 m = items[it];
    const uint32_t b = (uint32_t)m.y;
    const int len = m.z;
    for (int i = lane; i < len; i += 256) {
      int k[4];
      if (zw) {
        // the word-ordered copy: the item's topics are contiguous
#pragma unroll
        for (int u = 0; u < 4; ++u) k[u] = (i + 64 * u < len) ? zw[b + (uint32_t)(i + 64 * u)] : -1;
      } else {
        uint32_t tk[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) tk[u] = (i + 64 * u < len) ? perm[b + (uint32_t)(i + 64 * u)] : 0xFFFFFFFFu;
#pragma unroll
        for (int u = 0; u < 4; ++u) k[u] = tk[u] != 0xFFFFFFFFu ? z[tk[u]] : -1;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (k[u] >= 0) atomicAdd(&hist[k[u]], 1);
    }
    wave_lds_fence();
    int32_t h[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
      h[j] = hist[lane * C + j];
      hist[lane * C + j] = 0;
    }
    int32_t* row = buf + (int64_t)m.x * KP + lane * C;
    if (m.w == 0) {
#pragma unroll
      for (int j = 0; j < C; ++j) row[j] = h[j];
    } else {
#pragma unroll
      for (int j = 0; j < C; ++j)
        if (h[j]) atomicAdd(&row[j], h[j]);
    }
#pragma unroll
    for (int j = 0; j < C; ++j)
      if (h[j]) atomicAdd(&bs[lane * C + j], h[j]);
    wave_lds_fence();
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KP; i += 256) {
    const int v = bs[i];
    if (v != 0) atomicAdd(&bufsum[i], v);
  }
}

// ------------------------------------------------------------- launchers
template <int C>
static constexpr size_t sample_lds() { return (C <= 8 ? 11 : 10) * 64 * C * sizeof(int32_t); }
template <int C, int P, bool FROZEN>
static hipError_t launch_sample_t(const SampleParams& p, int blocks, hipStream_t st) {
  const size_t lds = sample_lds<C>();
  hipLaunchKernelGGL((k_sample<C, P, FROZEN>), dim3(blocks), dim3(256), lds, st, p);
  return hipGetLastError();
}

template <int C, int P, bool FROZEN>
static int occupancy_t() {
  int nb = 0;
  const size_t lds = sample_lds<C>();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sample<C, P, FROZEN>, 256, lds) !=
      hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}

#define LDA_DISPATCH_C(C_, FN, ...)                               \
  switch (C_) {                                                   \
    case 1: return FN<1, SAMPLE_P1, FROZEN>(__VA_ARGS__);         \
    case 2: return FN<2, SAMPLE_P2, FROZEN>(__VA_ARGS__);         \
    case 4: return FN<4, SAMPLE_P4, FROZEN>(__VA_ARGS__);         \
    case 8: return FN<8, SAMPLE_P8, FROZEN>(__VA_ARGS__);         \
    case 16: return FN<16, SAMPLE_P16, FROZEN>(__VA_ARGS__);      \
    default: break;                                               \
  }

// the half-wave kernel (K <= 128): topics per half-lane
int half_topics_per_lane(int K) { return K <= 32 ? 1 : (K <= 64 ? 2 : 4); }
template <int CH>
static constexpr size_t sample_half_lds() {
  constexpr int KH = 32 * CH, KP = KH < 64 ? 64 : KH;
  return (3 * KP + 16 * KH) * sizeof(int32_t);
}
template <int CH, bool FROZEN>
static hipError_t launch_half_t(const SampleParams& p, int blocks, hipStream_t st) {
  hipLaunchKernelGGL((k_sample_half<CH, SAMPLE_PH, FROZEN>), dim3(blocks), dim3(256), sample_half_lds<CH>(), st, p);
  return hipGetLastError();
}
template <int CH, bool FROZEN>
static int occupancy_half_t() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sample_half<CH, SAMPLE_PH, FROZEN>, 256,
                                                   sample_half_lds<CH>()) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}
int quarter_topics_per_lane(int K) { return K <= 16 ? 1 : (K <= 32 ? 2 : (K <= 64 ? 4 : 8)); }
template <int CH>
static constexpr size_t sample_quarter_lds() {
  constexpr int KQ = 16 * CH, KP = KQ < 64 ? 64 : KQ;
  return (3 * KP + 32 * KQ) * sizeof(int32_t);
}
template <int CH, bool FROZEN>
static hipError_t launch_quarter_t(const SampleParams& p, int blocks, hipStream_t st) {
  hipLaunchKernelGGL((k_sample_quarter<CH, SAMPLE_PQ, FROZEN>), dim3(blocks), dim3(256),
                     sample_quarter_lds<CH>(), st, p);
  return hipGetLastError();
}
template <int CH, bool FROZEN>
static int occupancy_quarter_t() {
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sample_quarter<CH, SAMPLE_PQ, FROZEN>, 256,
                                                   sample_quarter_lds<CH>()) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}
template <bool FROZEN>
static hipError_t launch_sample_c(int C, const SampleParams& p, int blocks, hipStream_t st, int half) {
  if (half == 2 && C <= 2) {
    switch (quarter_topics_per_lane(p.K)) {
      case 1: return launch_quarter_t<1, FROZEN>(p, blocks, st);
      case 2: return launch_quarter_t<2, FROZEN>(p, blocks, st);
      case 4: return launch_quarter_t<4, FROZEN>(p, blocks, st);
      default: return launch_quarter_t<8, FROZEN>(p, blocks, st);
    }
  }
  if (half == 1 && C <= 2) {
    switch (half_topics_per_lane(p.K)) {
      case 1: return launch_half_t<1, FROZEN>(p, blocks, st);
      case 2: return launch_half_t<2, FROZEN>(p, blocks, st);
      default: return launch_half_t<4, FROZEN>(p, blocks, st);
    }
  }
  LDA_DISPATCH_C(C, launch_sample_t, p, blocks, st)
  return hipErrorInvalidValue;
}
template <bool FROZEN>
static int occupancy_c(int C, int K, int half) {
  if (half == 2 && C <= 2) {
    switch (quarter_topics_per_lane(K)) {
      case 1: return occupancy_quarter_t<1, FROZEN>();
      case 2: return occupancy_quarter_t<2, FROZEN>();
      case 4: return occupancy_quarter_t<4, FROZEN>();
      default: return occupancy_quarter_t<8, FROZEN>();
    }
  }
  if (half == 1 && C <= 2) {
    switch (half_topics_per_lane(K)) {
      case 1: return occupancy_half_t<1, FROZEN>();
      case 2: return occupancy_half_t<2, FROZEN>();
      default: return occupancy_half_t<4, FROZEN>();
    }
  }
  LDA_DISPATCH_C(C, occupancy_t)
  return 1;
}

hipError_t launch_sample(int C, bool frozen, const SampleParams& p, int blocks, hipStream_t st,
                         int half) {
  return frozen ? launch_sample_c<true>(C, p, blocks, st, half)
                : launch_sample_c<false>(C, p, blocks, st, half);
}
int sample_blocks_per_cu(int C, bool frozen, int K, int half) {
  return frozen ? occupancy_c<true>(C, K, half) : occupancy_c<false>(C, K, half);
}

template <int C, int P, int R0, bool FROZEN>
static hipError_t launch_sparse_t(const SampleParams& p, int blocks, hipStream_t st) {
  const size_t lds = 12 * 64 * C * sizeof(int32_t);
  hipLaunchKernelGGL((k_sample_sparse<C, P, R0, FROZEN>), dim3(blocks), dim3(256), lds, st, p);
  return hipGetLastError();
}
template <int C, int P, int R0, bool FROZEN>
static int occupancy_sparse_t() {
  int nb = 0;
  const size_t lds = 12 * 64 * C * sizeof(int32_t);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sample_sparse<C, P, R0, FROZEN>, 256,
                                                   lds) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}
template <int C, int NS, int RB, bool FROZEN>
static size_t sparse_big_lds() {
  // {alpha, inv} table + per-wave 16-bit nd pairs; > 64 KiB at C = 64
  constexpr size_t lds = (2 * 64 * C + sb_waves<C>() * ((64 * C) >> kNdShift)) * sizeof(int32_t);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sample_big<C, NS, RB, FROZEN>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  }();
  (void)attr;
  return lds;
}
template <int C, int NS, int RB, bool FROZEN>
static hipError_t launch_sparse_big_rb(const SampleParams& p, int blocks, hipStream_t st) {
  const size_t lds = sparse_big_lds<C, NS, RB, FROZEN>();
  hipLaunchKernelGGL((k_sample_big<C, NS, RB, FROZEN>), dim3(blocks), dim3(64 * sb_waves<C>()),
                     lds, st, p);
  return hipGetLastError();
}
// rb: 0 for the default ring (SB_NS slots of SB_RB register rounds), else
// the short one (SB_NS_SHORT x SB_RB_SHORT) for short rows (the caller's
// choice, by timing both).  The same sums in the same order either way.
template <int C, bool FROZEN>
static hipError_t launch_sparse_big_t(const SampleParams& p, int blocks, hipStream_t st, int rb) {
  if (!FROZEN && rb != 0) return launch_sparse_big_rb<C, SB_NS_SHORT, SB_RB_SHORT, FROZEN>(p, blocks, st);
  return launch_sparse_big_rb<C, SB_NS, SB_RB, FROZEN>(p, blocks, st);
}
template <int C, bool FROZEN>
static int occupancy_sparse_big_t() {
  int nb = 0;
  const size_t lds = sparse_big_lds<C, SB_NS, SB_RB, FROZEN>();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sample_big<C, SB_NS, SB_RB, FROZEN>,
                                                   64 * sb_waves<C>(), lds) != hipSuccess)
    return 1;
  return nb > 0 ? nb : 1;
}
#define LDA_DISPATCH_SPARSE(C_, FN, ...)                            \
  switch (C_) {                                                     \
    case 1: return FN<1, SPARSE_P, 1, FROZEN>(__VA_ARGS__);         \
    case 2: return FN<2, SPARSE_P, 1, FROZEN>(__VA_ARGS__);         \
    case 4: return FN<4, SPARSE_P, SPARSE_R0, FROZEN>(__VA_ARGS__); \
    case 8: return FN<8, SPARSE_P, SPARSE_R0, FROZEN>(__VA_ARGS__); \
    case 16: return FN<16, SPARSE_P, SPARSE_R0, FROZEN>(__VA_ARGS__); \
    default: break;                                                 \
  }
template <bool FROZEN>
static hipError_t launch_sparse_c(int C, const SampleParams& p, int blocks, hipStream_t st, int rb) {
  if (C == 32) return launch_sparse_big_t<32, FROZEN>(p, blocks, st, rb);
  if (C == 64) return launch_sparse_big_t<64, FROZEN>(p, blocks, st, rb);
  LDA_DISPATCH_SPARSE(C, launch_sparse_t, p, blocks, st)
  return hipErrorInvalidValue;
}
template <bool FROZEN>
static int occupancy_sparse_c(int C) {
  if (C == 32) return occupancy_sparse_big_t<32, FROZEN>();
  if (C == 64) return occupancy_sparse_big_t<64, FROZEN>();
  LDA_DISPATCH_SPARSE(C, occupancy_sparse_t)
  return 1;
}
hipError_t launch_sample_sparse(int C, bool frozen, const SampleParams& p, int blocks,
                                hipStream_t st, int rb) {
  return frozen ? launch_sparse_c<true>(C, p, blocks, st, rb) : launch_sparse_c<false>(C, p, blocks, st, rb);
}
int sample_sparse_blocks_per_cu(int C, bool frozen) {
  return frozen ? occupancy_sparse_c<true>(C) : occupancy_sparse_c<false>(C);
}

int sample_waves_per_block(int C, bool sparse, int half) {
  if (sparse && C == 32) return sb_waves<32>();
  if (sparse && C == 64) return sb_waves<64>();
  if (!sparse && half == 1 && C <= 2) return 8;    // two range workers per wave
  if (!sparse && half == 2 && C <= 2) return 16;   // four range workers per wave
  return 4;
}

hipError_t launch_philox_draws(const int64_t* gtok, int64_t n, uint32_t c2, uint32_t c3, uint64_t seed,
                               uint32_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_philox_draws, dim3(blocks), dim3(256), 0, st, gtok, n, c2, c3, (uint32_t)seed,
                     (uint32_t)(seed >> 32), out);
  return hipGetLastError();
}

hipError_t launch_row_caps(const int32_t* nw, int64_t V, int32_t Kp, int32_t* caps, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((V + 3) / 4, 8192);
  hipLaunchKernelGGL(k_row_caps, dim3(blocks), dim3(256), 0, st, nw, V, Kp, caps);
  return hipGetLastError();
}

hipError_t launch_build_sparse(const int32_t* nw, int64_t V, int32_t Kp, const int64_t* row_off,
                               uint32_t* ent, int32_t* row_nnz, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((V + 3) / 4, 16384);
  switch (Kp / 64) {
    case 1: hipLaunchKernelGGL(k_build_sparse<1>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    case 2: hipLaunchKernelGGL(k_build_sparse<2>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    case 4: hipLaunchKernelGGL(k_build_sparse<4>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    case 8: hipLaunchKernelGGL(k_build_sparse<8>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    case 16: hipLaunchKernelGGL(k_build_sparse<16>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    case 32: hipLaunchKernelGGL(k_build_sparse<32>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    case 64: hipLaunchKernelGGL(k_build_sparse<64>, dim3(blocks), dim3(256), 0, st, nw, V, row_off, ent, row_nnz); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_build_packed(const int32_t* nw, int64_t V, int32_t Kp, uint16_t* nw16,
                               uint8_t* wide, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((V + 3) / 4, 16384);
  switch (Kp / 64) {
    case 1: hipLaunchKernelGGL(k_build_packed<1>, dim3(blocks), dim3(256), 0, st, nw, V, nw16, wide); break;
    case 2: hipLaunchKernelGGL(k_build_packed<2>, dim3(blocks), dim3(256), 0, st, nw, V, nw16, wide); break;
    case 4: hipLaunchKernelGGL(k_build_packed<4>, dim3(blocks), dim3(256), 0, st, nw, V, nw16, wide); break;
    case 8: hipLaunchKernelGGL(k_build_packed<8>, dim3(blocks), dim3(256), 0, st, nw, V, nw16, wide); break;
    case 16: hipLaunchKernelGGL(k_build_packed<16>, dim3(blocks), dim3(256), 0, st, nw, V, nw16, wide); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_apply_packed(int32_t* nw, int32_t* delta, int64_t V, int32_t Kp, uint16_t* nw16,
                               uint8_t* wide, const TopicTables& t, hipStream_t st) {
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((V + 3) / 4, 16384));
  switch (Kp / 64) {
    case 1: hipLaunchKernelGGL(k_apply_packed<1>, dim3(blocks), dim3(256), 0, st, nw, delta, V, nw16, wide, t); break;
    case 2: hipLaunchKernelGGL(k_apply_packed<2>, dim3(blocks), dim3(256), 0, st, nw, delta, V, nw16, wide, t); break;
    case 4: hipLaunchKernelGGL(k_apply_packed<4>, dim3(blocks), dim3(256), 0, st, nw, delta, V, nw16, wide, t); break;
    case 8: hipLaunchKernelGGL(k_apply_packed<8>, dim3(blocks), dim3(256), 0, st, nw, delta, V, nw16, wide, t); break;
    case 16: hipLaunchKernelGGL(k_apply_packed<16>, dim3(blocks), dim3(256), 0, st, nw, delta, V, nw16, wide, t); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_init_z(int32_t* z, int64_t n, int32_t K, int64_t token_base, uint32_t k0,
                         uint32_t k1, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_init_z, dim3(blocks), dim3(256), 0, st, z, n, K, token_base, k0, k1);
  return hipGetLastError();
}

hipError_t launch_count(const int32_t* words, const int32_t* z, int64_t n, int32_t Kp,
                        int32_t* delta, int32_t* dsum, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_count, dim3(blocks), dim3(256), Kp * sizeof(int32_t), st, words, z, n, Kp,
                     delta, dsum);
  return hipGetLastError();
}

#ifdef SB_X_DELTA_KERNEL
// measurement builds only: a token's count change from its topic before
// (zold) and after (z) the sampling pass, as the sampler's own atomics make it
__global__ __launch_bounds__(256) void k_delta_from_z(const int32_t* __restrict__ words,
                                                      const int32_t* __restrict__ zold,
                                                      const int32_t* __restrict__ z, int64_t n, int32_t Kp,
                                                      int32_t* __restrict__ delta) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int zo = zold[i], zn = z[i];
    if (zo != zn) {
      const int64_t rb = (int64_t)words[i] * Kp;
      atomicAdd(delta + rb + zo, -1);
      atomicAdd(delta + rb + zn, 1);
    }
  }
}
hipError_t launch_delta_from_z(const int32_t* words, const int32_t* zold, const int32_t* z, int64_t n,
                               int32_t Kp, int32_t* delta, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 16384);
  hipLaunchKernelGGL(k_delta_from_z, dim3(blocks), dim3(256), 0, st, words, zold, z, n, Kp, delta);
  return hipGetLastError();
}
#endif

hipError_t launch_apply(int32_t* nw, int32_t* delta, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  if (n4 <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_apply, dim3(blocks), dim3(256), 0, st, reinterpret_cast<int4*>(nw),
                     reinterpret_cast<int4*>(delta), n4);
  return hipGetLastError();
}

hipError_t launch_apply_cols(int32_t* nw, int32_t* delta, int64_t V, int32_t Kp, int32_t* dsum,
                             hipStream_t st) {
  const int64_t n4 = V * Kp / 4;
  if (n4 <= 0) return hipSuccess;
  const int kp4 = Kp / 4;                     // a power of two >= 16
  // the grid a multiple of kp4 threads (kp4 <= 1024: a multiple of 4 blocks
  // covers it), at most 512 blocks: ~Kp * 128 partial-sum atomics per apply
  const int unit = std::max(1, kp4 / 256);
  int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 512);
  blocks = std::max(unit, blocks / unit * unit);
  hipLaunchKernelGGL(k_apply_cols, dim3(blocks), dim3(256), 0, st, reinterpret_cast<int4*>(nw),
                     reinterpret_cast<int4*>(delta), n4, dsum, kp4);
  return hipGetLastError();
}

template <int C>
static hipError_t launch_apply_build_t(int32_t* nw, int32_t* delta, int64_t V, const int64_t* row_off,
                                       uint32_t* ent, int32_t* row_nnz, int32_t* dsum, hipStream_t st) {
  constexpr size_t lds = 4 * 64 * C * sizeof(int32_t);
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(&k_apply_build<C>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) == hipSuccess;
  }();
  (void)attr;
  const int blocks = (int)std::min<int64_t>((V + 3) / 4, 2048);
  hipLaunchKernelGGL(k_apply_build<C>, dim3(blocks), dim3(256), lds, st, nw, delta, V, row_off, ent, row_nnz,
                     dsum);
  return hipGetLastError();
}
hipError_t launch_apply_build(int32_t* nw, int32_t* delta, int64_t V, int32_t Kp, const int64_t* row_off,
                              uint32_t* ent, int32_t* row_nnz, int32_t* dsum, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  switch (Kp / 64) {
    case 1: return launch_apply_build_t<1>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    case 2: return launch_apply_build_t<2>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    case 4: return launch_apply_build_t<4>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    case 8: return launch_apply_build_t<8>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    case 16: return launch_apply_build_t<16>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    case 32: return launch_apply_build_t<32>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    case 64: return launch_apply_build_t<64>(nw, delta, V, row_off, ent, row_nnz, dsum, st);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_exch_pack(const int32_t* buf, int64_t cells, int32_t* packed, int32_t world,
                            int32_t* esc, int32_t cap, hipStream_t st, int32_t per_word) {
  const int64_t n4 = cells / 4;
  if (n4 <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
  if (per_word == 4)
    hipLaunchKernelGGL(k_exch_pack4, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const int4*>(buf), n4,
                       reinterpret_cast<uint32_t*>(packed), exch_bias4(world), exch_bias4_top(world), esc, cap);
  else
    hipLaunchKernelGGL(k_exch_pack, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const int4*>(buf), n4,
                       reinterpret_cast<uint2*>(packed), exch_bias0(world), exch_bias1(world), esc, cap);
  return hipGetLastError();
}

hipError_t launch_exch_unpack(const int32_t* packed, int64_t cells, int32_t* buf, int32_t world,
                              const int32_t* esc_all, int32_t cap, hipStream_t st, int32_t per_word) {
  const int64_t n4 = cells / 4;
  if (n4 > 0) {
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
    if (per_word == 4)
      hipLaunchKernelGGL(k_exch_unpack4, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const uint32_t*>(packed),
                         n4, reinterpret_cast<int4*>(buf), world * exch_bias4(world),
                         world * exch_bias4_top(world));
    else
      hipLaunchKernelGGL(k_exch_unpack, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const uint2*>(packed),
                         n4, reinterpret_cast<int4*>(buf), world * exch_bias0(world), world * exch_bias1(world));
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (!esc_all) return hipSuccess;      // no rank had an escape (lda_exchange_unpack_lists, list_cap 0)
  hipLaunchKernelGGL(k_exch_escapes, dim3(4 * world), dim3(256), 0, st, esc_all, cap, buf);
  return hipGetLastError();
}

hipError_t launch_counts_checksum(const int32_t* nw, const int32_t* nwsum, int32_t K, int32_t Kp, int64_t V,
                                  uint64_t* partial, int blocks, hipStream_t st) {
  hipLaunchKernelGGL(k_counts_checksum, dim3(blocks), dim3(256), 0, st, reinterpret_cast<const int4*>(nw),
                     V * Kp / 4, nwsum, K, Kp, V, partial);
  return hipGetLastError();
}

hipError_t launch_fold_delta(int32_t* dst, int32_t* src, int64_t n, hipStream_t st) {
  const int64_t n4 = n / 4;
  if (n4 <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 8192);
  hipLaunchKernelGGL(k_fold_delta, dim3(blocks), dim3(256), 0, st, reinterpret_cast<int4*>(dst),
                     reinterpret_cast<int4*>(src), n4);
  return hipGetLastError();
}

hipError_t launch_prepare_topics(int32_t* nwsum, int32_t* dsum, const double* alpha, double beta,
                                 double vbeta, int32_t K, int32_t Kp, float* alpha_f, float* inv,
                                 float* inv_m1, hipStream_t st) {
  hipLaunchKernelGGL(k_prepare_topics, dim3((Kp + 255) / 256), dim3(256), 0, st, nwsum, dsum, alpha,
                     beta, vbeta, K, Kp, alpha_f, inv, inv_m1);
  return hipGetLastError();
}

hipError_t launch_big_tables(const int32_t* nwsum, const float* alpha_f, const float* inv, const float* inv_m1,
                             int32_t K, int32_t Kp, float beta, const BigTables& t, hipStream_t st) {
  hipLaunchKernelGGL(k_big_tables, dim3(1), dim3(1024), 0, st, nwsum, alpha_f, inv, inv_m1, K, Kp, beta, t);
  return hipGetLastError();
}

hipError_t launch_doc_topics(const int32_t* z, const int64_t* doc_off, int64_t D, int32_t K,
                             int32_t Kp, int32_t* out, int accumulate, hipStream_t st) {
  if (D <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((D + 3) / 4, 4096);
  hipLaunchKernelGGL(k_doc_topics, dim3(blocks), dim3(256), 4 * Kp * sizeof(int32_t), st, z,
                     doc_off, D, K, Kp, out, accumulate);
  return hipGetLastError();
}

hipError_t launch_ll_docs(const int32_t* z, const int64_t* doc_off, int64_t D, const double* alpha,
                          double alpha_sum, int32_t K, int32_t Kp, double* partial, int blocks,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_ll_docs, dim3(blocks), dim3(256), 4 * Kp * sizeof(int32_t), st, z, doc_off, D,
                     alpha, alpha_sum, K, Kp, partial);
  return hipGetLastError();
}

hipError_t launch_ll_words(const int32_t* nw, int64_t V, int32_t K, int32_t Kp, double beta,
                           double* partial, unsigned long long* nonzero, int blocks,
                           hipStream_t st) {
  hipLaunchKernelGGL(k_ll_words, dim3(blocks), dim3(256), 0, st, nw, V, K, Kp, beta, partial,
                     nonzero);
  return hipGetLastError();
}

hipError_t launch_doc_hist(const int32_t* z, const int64_t* doc_off, int64_t D, int32_t K, int32_t Kp,
                           int32_t L, int32_t* len_hist, int32_t* topic_hist, hipStream_t st) {
  if (D <= 0) return hipSuccess;
  // >= 8 documents per wave, so the per-block flush is amortised
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((D + 31) / 32, 1024));
  const size_t lds = (4 * (size_t)Kp + DOC_HIST_LEN + (size_t)K * DOC_HIST_SMALL) * sizeof(int32_t);
  if (lds > 65536) {   // K > 1024: past the default dynamic LDS limit (160 KB per CU)
    const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(&k_doc_hist),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(k_doc_hist, dim3(blocks), dim3(256), lds, st, z, doc_off, D,
                     K, Kp, L, len_hist, topic_hist);
  return hipGetLastError();
}

hipError_t launch_count_hist(const int32_t* nw, int64_t V, int32_t K, int32_t Kp, int64_t max_count,
                             int32_t* hist, int32_t* overflow, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  // each block clears and flushes a 16 KB LDS histogram: >= 16 cells per
  // thread keep that off the small models' launch (4096 blocks of ~2 cells
  // each had taken 28 us at V = 5000, K = 500)
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((V * Kp + 4095) / 4096, 1024));
  hipLaunchKernelGGL(k_count_hist, dim3(blocks), dim3(256), 0, st, nw, V, K, Kp, max_count, hist,
                     overflow);
  return hipGetLastError();
}

hipError_t launch_row_stats(const int32_t* nw, int64_t V, int32_t K, int32_t Kp,
                            unsigned long long* out, hipStream_t st) {
  if (V <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((V + 3) / 4, 2048);
  hipLaunchKernelGGL(k_row_stats, dim3(blocks), dim3(256), 0, st, nw, V, K, Kp, out);
  return hipGetLastError();
}

hipError_t launch_infer_init(const int32_t* words, int32_t* z, int64_t n, const int32_t* nw,
                             int32_t K, int32_t Kp, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 3) / 4, 8192);
  hipLaunchKernelGGL(k_infer_init, dim3(blocks), dim3(256), 0, st, words, z, n, nw, K, Kp);
  return hipGetLastError();
}

hipError_t launch_word_hist(const int32_t* words, int64_t n, const PartSpans& ps, int64_t V,
                            uint32_t* cnt, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_word_hist, dim3(blocks), dim3(256), 0, st, words, n, ps, V, cnt);
  return hipGetLastError();
}

hipError_t launch_word_scatter(const int32_t* words, int64_t n, const PartSpans& ps, int64_t V,
                               uint32_t* cursor, uint32_t* perm, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_word_scatter, dim3(blocks), dim3(256), 0, st, words, n, ps, V, cursor, perm);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void k_zw_build(const uint32_t* __restrict__ perm, int64_t n,
                                                  const int32_t* __restrict__ z, uint32_t* __restrict__ zpos,
                                                  int32_t* __restrict__ zw) {
  for (int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (int64_t)gridDim.x * 256) {
    const uint32_t i = perm[j];
    zpos[i] = (uint32_t)j;
    zw[j] = z[i];
  }
}

hipError_t launch_zw_build(const uint32_t* perm, int64_t n, const int32_t* z, uint32_t* zpos, int32_t* zw,
                           hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 16384);
  hipLaunchKernelGGL(k_zw_build, dim3(blocks), dim3(256), 0, st, perm, n, z, zpos, zw);
  return hipGetLastError();
}

hipError_t launch_recount(int32_t Kp, const uint32_t* perm, const int32_t* zw, const int32_t* items, int32_t n_items,
                          const int32_t* z, int32_t* buf, int32_t* bufsum, int blocks, hipStream_t st) {
  if (n_items <= 0) return hipSuccess;
  blocks = std::max(1, std::min(blocks, (n_items + 3) / 4));
  const int4* it = reinterpret_cast<const int4*>(items);
  switch (Kp / 64) {
    case 1: hipLaunchKernelGGL(k_recount<1>, dim3(blocks), dim3(256), 0, st, perm, zw, it, n_items, z, buf, bufsum); break;
    case 2: hipLaunchKernelGGL(k_recount<2>, dim3(blocks), dim3(256), 0, st, perm, zw, it, n_items, z, buf, bufsum); break;
    case 4: hipLaunchKernelGGL(k_recount<4>, dim3(blocks), dim3(256), 0, st, perm, zw, it, n_items, z, buf, bufsum); break;
    case 8: hipLaunchKernelGGL(k_recount<8>, dim3(blocks), dim3(256), 0, st, perm, zw, it, n_items, z, buf, bufsum); break;
    case 16: hipLaunchKernelGGL(k_recount<16>, dim3(blocks), dim3(256), 0, st, perm, zw, it, n_items, z, buf, bufsum); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}


}  // namespace lda
