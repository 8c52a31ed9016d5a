// fetch_calib: known-byte read and write patterns for calibrating rocprofv3's
// FETCH_SIZE / WRITE_SIZE on gfx950 (MI355X_MICROARCH.md §HBM: "other access
// widths are uncalibrated: calibrate on a known byte count in your own access
// pattern").  Each kernel touches a known number of distinct bytes of a 4 GiB
// buffer (16x the Infinity Cache, so re-use is negligible):
//   k_stream4    coalesced 4 B/lane reads of the whole buffer
//   k_stream16   coalesced 16 B/lane reads of the whole buffer
//   k_round4     random 256 B rounds, 4 B/lane (the large-K sampler's entries)
//   k_row16      random 1 KiB rows, 16 B/lane (the dense sampler's K=512 rows)
//   k_row4x2     random 256 B rows, 4 B/lane (the dense sampler's K=128 rows)
//   k_write4     coalesced 4 B/lane stores of 1 GiB
//   k_atomic4    random 4 B int atomics, one per lane (the delta updates)
// Prints one JSON line {kernel: known bytes}; tools/fetch_calib.py joins it
// with the --pmc FETCH_SIZE / WRITE_SIZE summaries of the same program.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(256) void k_stream4(const uint32_t* __restrict__ a, int64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += a[i];
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_stream16(const uint4* __restrict__ a, int64_t n4, uint32_t* out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const uint4 v = a[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// one wave per iteration: a random 256 B-aligned round of the buffer
__global__ __launch_bounds__(256) void k_round4(const uint32_t* __restrict__ a, int64_t nrounds_buf,
                                                int64_t iters_per_wave, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  uint32_t acc = 0;
  for (int64_t it = 0; it < iters_per_wave; ++it) {
    const uint32_t r = mix32((uint32_t)(wave * iters_per_wave + it)) % (uint32_t)nrounds_buf;
    acc += a[(int64_t)r * 64 + lane];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// one wave per iteration: a random 1 KiB row, 16 B per lane
__global__ __launch_bounds__(256) void k_row16(const uint4* __restrict__ a, int64_t nrows_buf,
                                               int64_t iters_per_wave, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  uint32_t acc = 0;
  for (int64_t it = 0; it < iters_per_wave; ++it) {
    const uint32_t r = mix32((uint32_t)(wave * iters_per_wave + it) ^ 0x9e3779b9u) % (uint32_t)nrows_buf;
    const uint4 v = a[(int64_t)r * 64 + lane];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// one wave per iteration: a random 256 B row, 4 B per lane (2 topics per lane
// at K = 128 in 16-bit cells)
__global__ __launch_bounds__(256) void k_row4x2(const uint32_t* __restrict__ a, int64_t nrows_buf,
                                                int64_t iters_per_wave, uint32_t* out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  uint32_t acc = 0;
  for (int64_t it = 0; it < iters_per_wave; ++it) {
    const uint32_t r = mix32((uint32_t)(wave * iters_per_wave + it) ^ 0x85ebca6bu) % (uint32_t)nrows_buf;
    acc += a[(int64_t)r * 64 + lane];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_write4(uint32_t* __restrict__ a, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    a[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void k_atomic4(int32_t* __restrict__ a, int64_t ncells, int64_t per_thread) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (int64_t it = 0; it < per_thread; ++it) {
    const uint32_t c = mix32((uint32_t)(t * per_thread + it) ^ 0xc2b2ae35u) % (uint32_t)ncells;
    atomicAdd(a + c, 1);
  }
}

int main() {
  const int64_t bytes = int64_t(4) << 30;  // 4 GiB
  uint32_t* buf = nullptr;
  uint32_t* out = nullptr;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 1, bytes));
  CHECK(hipDeviceSynchronize());
  const int blocks = 256 * 16;
  const int64_t waves = (int64_t)blocks * 4;
  const int64_t n = bytes / 4;
  // random patterns: 2^26 x 256 B = 16 GiB of rounds requested over a 4 GiB
  // buffer would re-use lines; keep requests at 1/4 of the buffer so almost
  // every request is a distinct line (expected re-use < 12%)
  const int64_t rounds_buf = bytes / 256, rows_buf = bytes / 1024;
  const int64_t it_round = (bytes / 4 / 256) / waves;   // 1 GiB of 256 B rounds
  const int64_t it_row = (bytes / 4 / 1024) / waves;    // 1 GiB of 1 KiB rows
  const int64_t write_n = (int64_t(1) << 30) / 4;       // 1 GiB of stores
  const int64_t atom_per_thread = 64;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(k_stream4, dim3(blocks), dim3(256), 0, 0, buf, n, out);
    hipLaunchKernelGGL(k_stream16, dim3(blocks), dim3(256), 0, 0, reinterpret_cast<const uint4*>(buf), n / 4, out);
    hipLaunchKernelGGL(k_round4, dim3(blocks), dim3(256), 0, 0, buf, rounds_buf, it_round, out);
    hipLaunchKernelGGL(k_row16, dim3(blocks), dim3(256), 0, 0, reinterpret_cast<const uint4*>(buf), rows_buf, it_row, out);
    hipLaunchKernelGGL(k_row4x2, dim3(blocks), dim3(256), 0, 0, buf, rounds_buf, it_round, out);
    hipLaunchKernelGGL(k_write4, dim3(blocks), dim3(256), 0, 0, buf, write_n);
    hipLaunchKernelGGL(k_atomic4, dim3(blocks), dim3(256), 0, 0, reinterpret_cast<int32_t*>(buf), n, atom_per_thread);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
  }
  const double rd_round = (double)waves * it_round * 256, rd_row = (double)waves * it_row * 1024;
  printf("{\"k_stream4\": {\"read\": %.0f}, \"k_stream16\": {\"read\": %.0f}, "
         "\"k_round4\": {\"read_requested\": %.0f, \"read_distinct_expected\": %.0f}, "
         "\"k_row16\": {\"read_requested\": %.0f, \"read_distinct_expected\": %.0f}, "
         "\"k_row4x2\": {\"read_requested\": %.0f, \"read_distinct_expected\": %.0f}, "
         "\"k_write4\": {\"write\": %.0f}, \"k_atomic4\": {\"atomics\": %.0f, \"cells\": %.0f}}\n",
         (double)bytes, (double)bytes, rd_round,
         (double)rounds_buf * 256 * (1.0 - __builtin_exp(-rd_round / 256 / rounds_buf)), rd_row,
         (double)rows_buf * 1024 * (1.0 - __builtin_exp(-rd_row / 1024 / rows_buf)), rd_round,
         (double)rounds_buf * 256 * (1.0 - __builtin_exp(-rd_round / 256 / rounds_buf)), (double)write_n * 4,
         (double)blocks * 256 * atom_per_thread, (double)n);
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
