// Paired Montgomery multiplies: two independent mul29t column chains
// interleaved mad by mad, so no v_mad_u64_u32 result is read by the very next
// instruction (gfx950 inserts an s_nop after every dependent mad of a single
// chain).  Measures multiplies/s of 4 independent mul29t per iteration vs
// 2 x mul29t2, and checks that both give identical limbs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/field29.h"
using namespace qg;
using Q = F29<FqP>;

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ void mul29t2(const Q& a, const Q& b, const Q& c, const Q& d, Q& r1,
                                        Q& r2) {
  uint32_t m[9], n[9];
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      x = mad_vv(a.l[j], b.l[k - j], x);
      y = mad_vv(c.l[j], d.l[k - j], y);
      x = mad_vs(m[j], F29P<FqP>::P.v[k - j], x);
      y = mad_vs(n[j], F29P<FqP>::P.v[k - j], y);
    }
    x = mad_vv(a.l[k], b.l[0], x);
    y = mad_vv(c.l[k], d.l[0], y);
    m[k] = ((uint32_t)x * F29P<FqP>::INV) & M29;
    n[k] = ((uint32_t)y * F29P<FqP>::INV) & M29;
    x = mad_vs(m[k], F29P<FqP>::P.v[0], x);
    y = mad_vs(n[k], F29P<FqP>::P.v[0], y);
    x >>= 29;
    y >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
      x = mad_vv(a.l[j], b.l[k - j], x);
      y = mad_vv(c.l[j], d.l[k - j], y);
      x = mad_vs(m[j], F29P<FqP>::P.v[k - j], x);
      y = mad_vs(n[j], F29P<FqP>::P.v[k - j], y);
    }
    r1.l[k - 9] = (uint32_t)x & M29;
    r2.l[k - 9] = (uint32_t)y & M29;
    x >>= 29;
    y >>= 29;
  }
  r1.l[8] = (uint32_t)x;
  r2.l[8] = (uint32_t)y;
}
#else
__device__ void mul29t2(const Q& a, const Q& b, const Q& c, const Q& d, Q& r1, Q& r2);
#endif

__device__ Q load(const Fq* io, size_t i) { return to29(io[i & 1023]); }

template <int V>
__global__ void __launch_bounds__(256) k_tp(Fq* io, int iters) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Q a[4], b = load(io, i);
  for (int k = 0; k < 4; k++) a[k] = load(io, i + k + 1);
  for (int it = 0; it < iters; it++) {
    if constexpr (V == 0) {
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = mul29t(a[k], b);
    } else {
      mul29t2(a[0], b, a[1], b, a[0], a[1]);
      mul29t2(a[2], b, a[3], b, a[2], a[3]);
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 4; k++)
    for (int l = 0; l < 9; l++) s ^= a[k].l[l] * (2 * l + 1);
  if (s == 0x12345678u) io[i & 1023].v[0] = s;
}

__global__ void k_check(const Fq* io, uint32_t* out, int iters) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Q x = load(io, i), y = load(io, i + 7), b = load(io, i + 3);
  Q u = x, v = y;
  for (int it = 0; it < iters; it++) {
    x = mul29t(x, b);
    y = mul29t(y, b);
    mul29t2(u, b, v, b, u, v);
  }
  uint32_t bad = 0;
  for (int l = 0; l < 9; l++) bad |= (x.l[l] ^ u.l[l]) | (y.l[l] ^ v.l[l]);
  if (bad) atomicAdd(out, 1u);
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e = (x);                                               \
    if (e != hipSuccess) {                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

template <int V>
static void run(const char* name, Fq* io) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned blocks = 256 * 32;
  const int iters = 512;
  k_tp<V><<<blocks, 256>>>(io, 8);
  CK(hipEventRecord(a));
  k_tp<V><<<blocks, 256>>>(io, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"variant\": \"%s\", \"mul_per_s\": %.4g, \"ms\": %.3f}\n", name,
         (double)blocks * 256 * 4 * iters / (ms * 1e-3), ms);
}

int main() {
  Fq* io;
  uint32_t* bad;
  CK(hipMalloc(&io, 1024 * sizeof(Fq)));
  CK(hipMalloc(&bad, 4));
  CK(hipMemset(bad, 0, 4));
  Fq h[1024];
  uint64_t s = 0x1234567;
  for (int i = 0; i < 1024; i++) {
    for (int l = 0; l < 8; l++) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      h[i].v[l] = (uint32_t)(s >> 32);
    }
    h[i].v[7] &= 0x1fffffffu;
  }
  CK(hipMemcpy(io, h, sizeof(h), hipMemcpyHostToDevice));
  k_check<<<64, 256>>>(io, bad, 100);
  uint32_t nb = 0;
  CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  printf("{\"check_mismatch_threads\": %u}\n", nb);
  for (int rep = 0; rep < 2; rep++) {
    run<0>("mul29t_x4", io);
    run<1>("mul29t2_x2", io);
  }
  return nb ? 1 : 0;
}
