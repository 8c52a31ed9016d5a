// issue_peak.hip — measured instruction-issue peaks of one MI355X, the
// denominators of bench.py's issue-bound roofline.
//
// Every CU runs 32 waves (8 blocks of 256 threads) of independent chains:
//   salu: 8 independent s_add_u32 chains (scalar unit),
//   valu: 8 independent v_add_u32 chains (vector ALU, wave64),
//   mix:  both interleaved 1:1 (do the two issue in the same cycles?),
// and the chip-wide rate of wave-instructions per second is printed as JSON.
// hipcc --offload-arch=gfx950 -O3 tools/issue_peak.hip -o issue_peak
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHK(x)                                                                      \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                        \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

constexpr int kUnroll = 16;   // groups of 8 instructions per loop trip

__global__ __launch_bounds__(256) void k_salu(int iters, int seed, int* out) {
  int a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5,
      a6 = seed + 6, a7 = seed + 7;
  a0 = __builtin_amdgcn_readfirstlane(a0);
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      asm volatile(
          "s_add_u32 %0, %0, 3\n\ts_add_u32 %1, %1, 5\n\ts_add_u32 %2, %2, 7\n\ts_add_u32 %3, %3, 9\n\t"
          "s_add_u32 %4, %4, 11\n\ts_add_u32 %5, %5, 13\n\ts_add_u32 %6, %6, 15\n\ts_add_u32 %7, %7, 17"
          : "+s"(a0), "+s"(a1), "+s"(a2), "+s"(a3), "+s"(a4), "+s"(a5), "+s"(a6), "+s"(a7)
          :
          : "scc");
  }
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffff && threadIdx.x == 0) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_valu(int iters, int seed, int* out) {
  int a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
      a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      asm volatile(
          "v_add_u32 %0, %0, 3\n\tv_add_u32 %1, %1, 5\n\tv_add_u32 %2, %2, 7\n\tv_add_u32 %3, %3, 9\n\t"
          "v_add_u32 %4, %4, 11\n\tv_add_u32 %5, %5, 13\n\tv_add_u32 %6, %6, 15\n\tv_add_u32 %7, %7, 17"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
  }
  if (a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 == 0x7fffffff) out[0] = 1;
}

__global__ __launch_bounds__(256) void k_mix(int iters, int seed, int* out) {
  int s0 = __builtin_amdgcn_readfirstlane(seed), s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
  int v0 = seed + threadIdx.x, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < kUnroll; ++u)
      asm volatile(
          "s_add_u32 %0, %0, 3\n\tv_add_u32 %4, %4, 3\n\ts_add_u32 %1, %1, 5\n\tv_add_u32 %5, %5, 5\n\t"
          "s_add_u32 %2, %2, 7\n\tv_add_u32 %6, %6, 7\n\ts_add_u32 %3, %3, 9\n\tv_add_u32 %7, %7, 9"
          : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3)
          :
          : "scc");
  }
  if (s0 + s1 + s2 + s3 + v0 + v1 + v2 + v3 == 0x7fffffff) out[0] = 1;
}

template <typename F>
static int run(const char* name, F kern, int cus, double* rate) {
  int* out = nullptr;
  CHK(hipMalloc(&out, 4));
  const int iters = 4000, blocks = cus * 8;          // 32 waves per CU
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters / 10, 1, out);   // warm-up
  CHK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; ++r) {
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, iters, 1, out);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  const double waves = (double)blocks * 4.0;
  const double instr = waves * (double)iters * kUnroll * 8.0;   // the kernel's counted instructions
  *rate = instr / (best * 1e-3);
  fprintf(stderr, "%s: %.3f ms, %.4g wave-instructions/s\n", name, best, *rate);
  CHK(hipFree(out));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  double salu = 0, valu = 0, mix = 0;
  if (run("salu", k_salu, p.multiProcessorCount, &salu)) return 1;
  if (run("valu", k_valu, p.multiProcessorCount, &valu)) return 1;
  if (run("mix", k_mix, p.multiProcessorCount, &mix)) return 1;
  printf("{\"device\": \"%s\", \"cus\": %d, \"salu_per_s\": %.6g, \"valu_per_s\": %.6g, "
         "\"mix_per_s\": %.6g, \"waves_per_cu\": 32, \"note\": \"chip-wide wave-instructions per second, "
         "independent s_add_u32 / v_add_u32 chains; mix = SALU and VALU interleaved 1:1 (sum of both)\"}\n",
         p.gcnArchName, p.multiProcessorCount, salu, valu, mix);
  return 0;
}
