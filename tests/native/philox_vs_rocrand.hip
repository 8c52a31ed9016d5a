// The sampler's device RNG (liblda_mi355x.so, lda_philox_draws: word 0 of
// Philox4x32-10 with counter {gtok lo, gtok hi, sweep, stream} and key = the
// seed) against rocRAND's philox4x32_10 on the same GPU.
// rocRAND's engine with seed S, subsequence sweep | stream << 32 and offset
// 4 * gtok sits on counter {gtok lo, gtok hi, sweep, stream}, key {S lo, S hi},
// and its next number is word 0 of that block (offsets fit 64 bits for
// gtok < 2^62).  Prints one line and exits 0
// when every draw agrees.
#include <hip/hip_runtime.h>
#include <rocrand/rocrand_kernel.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#include "lda_mi355x.h"

__global__ void k_rocrand(const int64_t* gtok, int n, unsigned long long seed, uint32_t c2, uint32_t c3,
                          uint32_t* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  rocrand_state_philox4x32_10 st;
  const unsigned long long sub = (unsigned long long)c2 | ((unsigned long long)c3 << 32);
  rocrand_init(seed, sub, 4ull * (unsigned long long)gtok[i], &st);
  out[i] = rocrand(&st);
}

int main() {
  std::vector<int64_t> g;
  for (int64_t i = 0; i < 4096; ++i) g.push_back(i);
  const int64_t big[] = {(1ll << 31) - 1, 1ll << 31, (1ll << 32) - 1, 1ll << 32, (1ll << 32) + 12345,
                         2200000000ll, 10000000000ll, (1ll << 40) + 7, (1ll << 61) + 3};
  for (int64_t b : big)
    for (int64_t d = 0; d < 64; ++d) g.push_back(b + d);
  const unsigned long long seeds[] = {0ull, 1ull, 42ull, 20261015ull, 0xFFFFFFFFull, 0x123456789ABCDEFull};
  const uint32_t sweeps[] = {0u, 1u, 999u, 0xFFFFFFFFu};
  const uint32_t streams[] = {0u, 1u, 2u};
  const int n = (int)g.size();
  int64_t* dg = nullptr;
  uint32_t* dout = nullptr;
  if (hipMalloc(&dg, sizeof(int64_t) * n) != hipSuccess || hipMalloc(&dout, sizeof(uint32_t) * n) != hipSuccess ||
      hipMemcpy(dg, g.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice) != hipSuccess) {
    fprintf(stderr, "hip setup failed\n");
    return 2;
  }
  std::vector<uint32_t> a(n), b(n);
  long checked = 0, bad = 0;
  for (unsigned long long seed : seeds)
    for (uint32_t c2 : sweeps)
      for (uint32_t c3 : streams) {
        if (lda_philox_draws(seed, c2, c3, g.data(), n, a.data()) != LDA_OK) {
          fprintf(stderr, "lda_philox_draws: %s\n", lda_last_error());
          return 2;
        }
        hipLaunchKernelGGL(k_rocrand, dim3((n + 255) / 256), dim3(256), 0, 0, dg, n, seed, c2, c3, dout);
        if (hipMemcpy(b.data(), dout, sizeof(uint32_t) * n, hipMemcpyDeviceToHost) != hipSuccess) return 2;
        for (int i = 0; i < n; ++i) {
          ++checked;
          if (a[i] != b[i] && bad++ < 5)
            fprintf(stderr, "mismatch seed %llu sweep %u stream %u gtok %lld: %08x vs rocrand %08x\n", seed,
                    c2, c3, (long long)g[i], a[i], b[i]);
        }
      }
  (void)hipFree(dg);
  (void)hipFree(dout);
  printf("{\"checked\": %ld, \"mismatches\": %ld}\n", checked, bad);
  return bad ? 1 : 0;
}
