// Random row-gather throughput by row size (micro benchmark).  The MSM
// accumulate gathers one SRS table row per digit (2.18e8 rows per 2^24 MSM);
// this measures how many random rows per second the chip serves for rows of
// 128 B (reading 80 B of them, as msm_pt_load does, or all 128 B), 64 B and
// 32 B, over a 16 GiB table (far beyond L2 / MALL), with one gather per lane
// (maximal memory-level parallelism) and with G gathers per lane issued back
// to back.  hipcc --offload-arch=gfx950 -O3 -o micro/gather_bench micro/gather_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t i) {
  uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  return h;
}

// ROW bytes per row, LOADS 16-B loads from the row start (the 128-B / 80-B
// case loads words 0,1,2,3,6 like msm_pt_load: x, y and the top limbs)
template <int ROW, int LOADS, int G>
__global__ void __launch_bounds__(256) k_gather(const uint4* __restrict__ table, uint64_t rows,
                                               uint64_t n, uint32_t* __restrict__ sink) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i * G >= n) return;
  uint32_t s = 0;
  uint4 v[G][LOADS];
#pragma unroll
  for (int g = 0; g < G; g++) {
    const uint64_t r = mix(i * G + g) % rows;
    const uint4* p = table + r * (ROW / 16);
#pragma unroll
    for (int l = 0; l < LOADS; l++) v[g][l] = p[(ROW == 128 && LOADS == 5 && l == 4) ? 6 : l];
  }
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int l = 0; l < LOADS; l++) s ^= v[g][l].x ^ v[g][l].y ^ v[g][l].z ^ v[g][l].w;
  sink[i & ((1u << 20) - 1)] ^= s;
}

// cooperative: LPR lanes per row, each loads one 16-B word of it (the row's
// words in one coalesced request); a lane then owns 16 B of the row
template <int ROW, int LPR>
__global__ void __launch_bounds__(256) k_gather_coop(const uint4* __restrict__ table, uint64_t rows,
                                                    uint64_t n, uint32_t* __restrict__ sink) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t g = t / LPR;  // gather index
  if (g >= n) return;
  const uint64_t r = mix(g) % rows;
  const uint4 v = table[r * (ROW / 16) + (t % LPR)];
  sink[t & ((1u << 20) - 1)] ^= v.x ^ v.y ^ v.z ^ v.w;
}

template <int ROW, int LPR>
static void run_coop(const uint4* table, uint64_t bytes, uint32_t* sink, const char* name) {
  const uint64_t rows = bytes / ROW;
  const uint64_t n = 1ull << 27;  // gathers
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned blocks = (unsigned)((n * LPR + 255) / 256);
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_gather_coop<ROW, LPR>), dim3(blocks), dim3(256), 0, 0, table, rows, n,
                       sink);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep == 2)
      printf("%-28s rows=%.3g  %.3f ms  %.3g rows/s  %.0f GB/s of loaded bytes\n", name,
             (double)rows, ms, n / (ms * 1e-3), n * LPR * 16.0 / (ms * 1e-3) / 1e9);
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

template <int ROW, int LOADS, int G>
static void run(const uint4* table, uint64_t bytes, uint32_t* sink, const char* name) {
  const uint64_t rows = bytes / ROW;
  const uint64_t n = 1ull << 27;  // gathers
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned blocks = (unsigned)((n / G + 255) / 256);
  for (int rep = 0; rep < 3; rep++) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((k_gather<ROW, LOADS, G>), dim3(blocks), dim3(256), 0, 0, table, rows, n,
                       sink);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep == 2)
      printf("%-28s rows=%.3g  %.3f ms  %.3g rows/s  %.0f GB/s of loaded bytes  %.0f GB/s of rows\n",
             name, (double)rows, ms, n / (ms * 1e-3), n * LOADS * 16.0 / (ms * 1e-3) / 1e9,
             n * (double)ROW / (ms * 1e-3) / 1e9);
  }
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
}

int main() {
  const uint64_t bytes = 16ull << 30;
  uint4* table;
  uint32_t* sink;
  CK(hipMalloc(&table, bytes));
  CK(hipMalloc(&sink, 4u << 20));
  CK(hipMemset(table, 0x5a, bytes));
  CK(hipMemset(sink, 0, 4u << 20));
  CK(hipDeviceSynchronize());
  run<128, 5, 1>(table, bytes, sink, "128B row, 80B loaded, G=1");
  run<128, 8, 1>(table, bytes, sink, "128B row, 128B loaded, G=1");
  run<64, 4, 1>(table, bytes, sink, "64B row, 64B loaded, G=1");
  run<32, 2, 1>(table, bytes, sink, "32B row, 32B loaded, G=1");
  run<128, 5, 4>(table, bytes, sink, "128B row, 80B loaded, G=4");
  run<64, 4, 4>(table, bytes, sink, "64B row, 64B loaded, G=4");
  run_coop<128, 8>(table, bytes, sink, "coop 8 lanes x 16B of 128B");
  run_coop<128, 4>(table, bytes, sink, "coop 4 lanes x 16B of 128B");
  run_coop<64, 4>(table, bytes, sink, "coop 4 lanes x 16B of 64B");
  run<128, 5, 1>(table, 4ull << 30, sink, "128B row 80B, 4 GiB table");
  run<128, 5, 1>(table, 8ull << 30, sink, "128B row 80B, 8 GiB table");
  run_coop<128, 8>(table, 2ull << 30, sink, "coop 8x16B, 2 GiB table");
  run<128, 5, 1>(table, bytes / 8, sink, "128B row 80B, 2 GiB table");
  run<64, 4, 1>(table, bytes / 8, sink, "64B row, 2 GiB table");
  CK(hipFree(table));
  CK(hipFree(sink));
  return 0;
}
