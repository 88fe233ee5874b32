// 9 x 29-bit-limb Montgomery multiplication (R = 2^261) vs the 8 x 32-bit FIPS
// multiply, on gfx950.  With 29-bit limbs a column of 18 partial products
// stays below 2^63, so every product is a single v_mad_u64_u32 into a 64-bit
// accumulator — no carry-out / v_addc per product, no VCC hazards.
// Checks: mul29(x, y) == x * y * 2^-261 mod p (via the FIPS multiply), and
// throughput / single-wave latency of both.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/field.h"
using namespace qg;

struct F29 {
  uint32_t l[9];
};

__constant__ uint32_t P29[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                                0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
static constexpr uint32_t INV29 = 0x4866389u;
static constexpr uint32_t M29 = (1u << 29) - 1;

__device__ __forceinline__ F29 mul29(const F29& a, const F29& b) {
  constexpr uint32_t P[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                             0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      acc += (uint64_t)m[j] * P[k - j];
    }
    acc += (uint64_t)a.l[k] * b.l[0];
    m[k] = ((uint32_t)acc * INV29) & M29;
    acc += (uint64_t)m[k] * P[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      acc += (uint64_t)m[j] * P[k - j];
    }
    r.l[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// split accumulators: a*b chain and m*p chain per column (NA = 2), or each
// of them split again by parity of j (NA = 4); merged at the column end
template <int NA>
__device__ __forceinline__ F29 mul29s(const F29& a, const F29& b) {
  constexpr uint32_t P[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                             0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
  uint32_t m[9];
  F29 r;
  uint64_t A = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint64_t ab[2] = {0, 0}, mp[2] = {0, 0};
    const int jlo = k > 8 ? k - 8 : 0;
    const int jab = k < 8 ? k : 8;        // a*b: j in [jlo, jab]
    const int jmp = k < 9 ? k - 1 : 8;    // m*p: j in [jlo, jmp] (m_k not known yet)
#pragma unroll
    for (int j = jlo; j <= jab; j++) ab[NA == 4 ? (j & 1) : 0] += (uint64_t)a.l[j] * b.l[k - j];
#pragma unroll
    for (int j = jlo; j <= jmp; j++) mp[NA == 4 ? (j & 1) : 0] += (uint64_t)m[j] * P[k - j];
    A += ab[0] + ab[1] + mp[0] + mp[1];
    if (k < 9) {
      m[k] = ((uint32_t)A * INV29) & M29;
      A += (uint64_t)m[k] * P[0];
    } else {
      r.l[k - 9] = (uint32_t)A & M29;
    }
    A >>= 29;
  }
  r.l[8] = (uint32_t)A;
  return r;
}

// one accumulation chain per column, kept by inline asm (the compiler cannot
// re-associate it into split chains merged by 64-bit adds); p limbs in SGPRs
__device__ __forceinline__ uint64_t mad_asm(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ uint64_t mad_asm_s(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(cc) : "v"(a), "s"(b), "v"(c));
  return r;
}
__device__ __forceinline__ F29 mul29a(const F29& a, const F29& b) {
  constexpr uint32_t P[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                             0x2db40c0u,  0xa6e141u,  0xe5c2634u,  0x30644eu};
  uint32_t m[9];
  F29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      acc = mad_asm(a.l[j], b.l[k - j], acc);
      acc = mad_asm_s(m[j], P[k - j], acc);
    }
    acc = mad_asm(a.l[k], b.l[0], acc);
    m[k] = ((uint32_t)acc * INV29) & M29;
    acc = mad_asm_s(m[k], P[0], acc);
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
      acc = mad_asm(a.l[j], b.l[k - j], acc);
      acc = mad_asm_s(m[j], P[k - j], acc);
    }
    r.l[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

__device__ __forceinline__ F29 to29(const Fq& x) {
  F29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int lo = 29 * i, w = lo >> 5, s = lo & 31;
    uint64_t v = x.v[w];
    if (w + 1 < 8) v |= (uint64_t)x.v[w + 1] << 32;
    r.l[i] = (uint32_t)(v >> s) & M29;
  }
  return r;
}

// normalized limbs (< 2^29, top < 2^29) -> 8 x 32 (value < 2^256 assumed)
__device__ __forceinline__ Fq from29(const F29& a) {
  Fq r;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int lo = 32 * w, i = lo / 29, s = lo % 29;
    uint64_t v = (uint64_t)a.l[i] >> s;
    if (i + 1 < 9) v |= (uint64_t)a.l[i + 1] << (29 - s);
    if (i + 2 < 9 && 58 - s < 64) v |= (uint64_t)a.l[i + 2] << (58 - s);
    r.v[w] = (uint32_t)v;
  }
  return r;
}

template <int V>
__device__ __forceinline__ void mulv(Fq& a, F29& a29, const Fq& b, const F29& b29) {
  if constexpr (V == 0) a = a * b;
  else if constexpr (V == 1) a29 = mul29(a29, b29);
  else if constexpr (V == 2) a29 = mul29s<2>(a29, b29);
  else if constexpr (V == 3) a29 = mul29s<4>(a29, b29);
  else a29 = mul29a(a29, b29);
}

template <int V>
__global__ void __launch_bounds__(256) k_tp(Fq* io, int iters) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Fq a[4], b = io[i & 1023];
  F29 a29[4], b29 = to29(b);
  for (int k = 0; k < 4; k++) {
    a[k] = io[(i + k + 1) & 1023];
    a29[k] = to29(a[k]);
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 4; k++) mulv<V>(a[k], a29[k], b, b29);
  }
  uint32_t s = 0;
  for (int k = 0; k < 4; k++)
    for (int l = 0; l < 8; l++) s ^= a[k].v[l] ^ a29[k].l[l];
  if (s == 0x12345678u) io[i & 1023].v[0] = s;
}

template <int V>
__global__ void __launch_bounds__(256) k_tp1(Fq* io, int iters) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Fq a = io[(i + 1) & 1023], b = io[i & 1023];
  F29 a29 = to29(a), b29 = to29(b);
  for (int it = 0; it < iters; it++) mulv<V>(a, a29, b, b29);
  uint32_t s = 0;
  for (int l = 0; l < 8; l++) s ^= a.v[l] ^ a29.l[l];
  if (s == 0x12345678u) io[i & 1023].v[0] = s;
}

template <int V>
__global__ void k_lat(Fq* io, int iters) {
  Fq a = io[threadIdx.x], b = io[threadIdx.x + 1];
  F29 a29 = to29(a), b29 = to29(b);
  for (int it = 0; it < iters; it++) mulv<V>(a, a29, b, b29);
  io[2048 + threadIdx.x] = V == 0 ? a : from29(a29);
}

// out29 = canonical(mul29(x, y)); ref = (x * y) * 2^251 (FIPS, R = 2^256) = x y 2^-261
__global__ void k_check(const Fq* x, const Fq* y, Fq* o29, Fq* oref, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fq z = from29(mul29(to29(x[i]), to29(y[i])));
  Fq z2 = from29(mul29s<2>(to29(x[i]), to29(y[i])));
  Fq z4 = from29(mul29s<4>(to29(x[i]), to29(y[i])));
  Fq za = from29(mul29a(to29(x[i]), to29(y[i])));
  for (int l = 0; l < 8; l++)
    if (z2.v[l] != z.v[l] || z4.v[l] != z.v[l] || za.v[l] != z.v[l]) z.v[0] ^= 1;  // poison
  // z < 2p: reduce once
  uint32_t t[8];
  for (int l = 0; l < 8; l++) t[l] = z.v[l];
  reduce_once<FqP>(t);
  for (int l = 0; l < 8; l++) z.v[l] = t[l];
  o29[i] = z;
  Fq c = Fq::zero();
  c.v[7] = 0x08000000u;  // 2^251
  oref[i] = (x[i] * y[i]) * c;
}

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);             \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

template <int V>
static void run(const char* name, Fq* io) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned blocks = 256 * 16;
  const int iters = 1024;
  k_tp<V><<<blocks, 256>>>(io, 16);
  CK(hipEventRecord(a));
  k_tp<V><<<blocks, 256>>>(io, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  double tp = (double)blocks * 256 * 4 * iters / (ms * 1e-3);
  k_tp1<V><<<blocks, 256>>>(io, 16);
  CK(hipEventRecord(a));
  k_tp1<V><<<blocks, 256>>>(io, iters);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  double tp1 = (double)blocks * 256 * iters / (ms * 1e-3);
  k_lat<V><<<1, 64>>>(io, 16);
  CK(hipEventRecord(a));
  k_lat<V><<<1, 64>>>(io, 4096);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"variant\": \"%s\", \"mul_per_s_4chains\": %.4g, \"mul_per_s_1chain\": %.4g, \"latency_ns\": %.1f}\n",
         name, tp, tp1, ms * 1e6 / 4096);
}

int main() {
  const int n = 1 << 16;
  Fq *io, *x, *y, *o29, *oref;
  CK(hipMalloc(&io, 4096 * sizeof(Fq)));
  CK(hipMalloc(&x, n * sizeof(Fq)));
  CK(hipMalloc(&y, n * sizeof(Fq)));
  CK(hipMalloc(&o29, n * sizeof(Fq)));
  CK(hipMalloc(&oref, n * sizeof(Fq)));
  Fq* h = (Fq*)malloc(n * sizeof(Fq));
  uint64_t s = 0x1234567;
  for (int i = 0; i < n; i++) {
    for (int l = 0; l < 8; l++) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      h[i].v[l] = (uint32_t)(s >> 32);
    }
    h[i].v[7] &= 0x1fffffffu;
    if (i < 4)
      for (int l = 0; l < 8; l++) h[i].v[l] = (i == 0) ? 0 : FqP::P[l] - (l == 0 ? (uint32_t)i : 0u);
  }
  CK(hipMemcpy(x, h, n * sizeof(Fq), hipMemcpyHostToDevice));
  for (int i = 0; i < n; i++) h[i].v[0] ^= 0x9e3779b9u;
  CK(hipMemcpy(y, h, n * sizeof(Fq), hipMemcpyHostToDevice));
  CK(hipMemcpy(io, h, 4096 * sizeof(Fq), hipMemcpyHostToDevice));
  k_check<<<n / 256, 256>>>(x, y, o29, oref, n);
  CK(hipDeviceSynchronize());
  Fq* r0 = (Fq*)malloc(n * sizeof(Fq));
  Fq* r1 = (Fq*)malloc(n * sizeof(Fq));
  CK(hipMemcpy(r0, o29, n * sizeof(Fq), hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1, oref, n * sizeof(Fq), hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < n; i++)
    for (int l = 0; l < 8; l++)
      if (r0[i].v[l] != r1[i].v[l]) {
        bad++;
        break;
      }
  printf("{\"check\": {\"mul29_mismatch\": %d}}\n", bad);
  run<0>("fips_asm_32", io);
  run<1>("mont29_9limb", io);
  run<2>("mont29_split2", io);
  run<3>("mont29_split4", io);
  run<4>("mont29_asm_1chain", io);
  return bad ? 1 : 0;
}
