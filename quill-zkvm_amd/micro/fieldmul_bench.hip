// Field-multiplication microbenchmark for gfx950: CIOS (C) vs FIPS with an
// inline-asm v_mad_u64_u32/v_addc multiply-accumulate, single and dual
// accumulator.  Reports throughput (all CUs busy) and single-wave latency,
// and cross-checks the variants bit-for-bit on random inputs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../csrc/field.h"
using namespace qg;

__device__ __forceinline__ void mac96(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t r;
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %4\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "=&v"(r), "+v"(hi) : "v"(a), "v"(b), "v"(acc) : "vcc");
  acc = r;
}

template <class C>
__device__ __forceinline__ Fp<C> mul_fips(const Fp<C>& a, const Fp<C>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0;
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      mac96(acc, hi, a.v[j], b.v[k - j]);
      mac96(acc, hi, m[j], C::P[k - j]);
    }
    mac96(acc, hi, a.v[k], b.v[0]);
    m[k] = (uint32_t)acc * C::INV;
    mac96(acc, hi, m[k], C::P[0]);
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int j = k - 7; j < 8; j++) {
      mac96(acc, hi, a.v[j], b.v[k - j]);
      mac96(acc, hi, m[j], C::P[k - j]);
    }
    t[k - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
  }
  t[7] = (uint32_t)acc;
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  reduce_once<C>(r.v);
  return r;
}

// two independent accumulators (a*b products / m*P products), merged per column
template <class C>
__device__ __forceinline__ Fp<C> mul_fips2(const Fp<C>& a, const Fp<C>& b) {
  uint32_t m[8], t[8];
  uint64_t acc = 0, acc2 = 0;
  uint32_t hi = 0, hi2 = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      mac96(acc, hi, a.v[j], b.v[k - j]);
      mac96(acc2, hi2, m[j], C::P[k - j]);
    }
    mac96(acc, hi, a.v[k], b.v[0]);
    // merge acc2 into acc (96-bit add)
    {
      uint64_t s = acc + acc2;
      hi += hi2 + (s < acc ? 1u : 0u);
      acc = s;
    }
    m[k] = (uint32_t)acc * C::INV;
    mac96(acc, hi, m[k], C::P[0]);
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
    acc2 = 0;
    hi2 = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int j = k - 7; j < 8; j++) {
      mac96(acc, hi, a.v[j], b.v[k - j]);
      mac96(acc2, hi2, m[j], C::P[k - j]);
    }
    {
      uint64_t s = acc + acc2;
      hi += hi2 + (s < acc ? 1u : 0u);
      acc = s;
    }
    t[k - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)hi << 32);
    hi = 0;
    acc2 = 0;
    hi2 = 0;
  }
  t[7] = (uint32_t)acc;
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  reduce_once<C>(r.v);
  return r;
}

template <int V>
__device__ __forceinline__ Fq mulv(const Fq& a, const Fq& b) {
  if constexpr (V == 0) return a * b;
  else if constexpr (V == 1) return mul_fips(a, b);
  else return mul_fips2(a, b);
}

template <int V>
__global__ void __launch_bounds__(256) k_tp(Fq* io, int iters) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Fq a[4], b = io[i & 1023];
  for (int k = 0; k < 4; k++) a[k] = io[(i + k + 1) & 1023];
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = mulv<V>(a[k], b);
  }
  Fq s = a[0] + a[1] + a[2] + a[3];
  if (s.v[0] == 0x12345678u) io[i & 1023] = s;
}

template <int V>
__global__ void k_lat(Fq* io, int iters) {
  Fq a = io[threadIdx.x], b = io[threadIdx.x + 1];
  for (int it = 0; it < iters; it++) a = mulv<V>(a, b);
  io[2048 + threadIdx.x] = a;
}

template <int V>
__global__ void k_check(const Fq* x, const Fq* y, Fq* out, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = mulv<V>(x[i], y[i]);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

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
  k_lat<V><<<1, 64>>>(io, 16);
  CK(hipEventRecord(a));
  k_lat<V><<<1, 64>>>(io, 4096);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  double lat_ns = ms * 1e6 / 4096;
  printf("{\"variant\": \"%s\", \"mul_per_s\": %.4g, \"latency_ns\": %.1f}\n", name, tp, lat_ns);
}

int main() {
  const int n = 1 << 16;
  Fq *io, *x, *y, *o0, *o1, *o2;
  CK(hipMalloc(&io, 4096 * sizeof(Fq)));
  CK(hipMalloc(&x, n * sizeof(Fq)));
  CK(hipMalloc(&y, n * sizeof(Fq)));
  CK(hipMalloc(&o0, n * sizeof(Fq)));
  CK(hipMalloc(&o1, n * sizeof(Fq)));
  CK(hipMalloc(&o2, n * sizeof(Fq)));
  // random reduced inputs (< p): top limb masked below p's top limb
  Fq* h = (Fq*)malloc(n * sizeof(Fq));
  uint64_t s = 0x1234567;
  for (int i = 0; i < n; i++) {
    for (int l = 0; l < 8; l++) {
      s = s * 6364136223846793005ull + 1442695040888963407ull;
      h[i].v[l] = (uint32_t)(s >> 32);
    }
    h[i].v[7] &= 0x1fffffffu;
    if (i < 4) for (int l = 0; l < 8; l++) h[i].v[l] = (i == 0) ? 0 : FqP::P[l] - (l == 0 ? (uint32_t)i : 0u);
  }
  CK(hipMemcpy(x, h, n * sizeof(Fq), hipMemcpyHostToDevice));
  for (int i = 0; i < n; i++) h[i].v[0] ^= 0x9e3779b9u;
  CK(hipMemcpy(y, h, n * sizeof(Fq), hipMemcpyHostToDevice));
  CK(hipMemcpy(io, h, 4096 * sizeof(Fq), hipMemcpyHostToDevice));
  k_check<0><<<n / 256, 256>>>(x, y, o0, n);
  k_check<1><<<n / 256, 256>>>(x, y, o1, n);
  k_check<2><<<n / 256, 256>>>(x, y, o2, n);
  CK(hipDeviceSynchronize());
  Fq* r0 = (Fq*)malloc(n * sizeof(Fq));
  Fq* r1 = (Fq*)malloc(n * sizeof(Fq));
  Fq* r2 = (Fq*)malloc(n * sizeof(Fq));
  CK(hipMemcpy(r0, o0, n * sizeof(Fq), hipMemcpyDeviceToHost));
  CK(hipMemcpy(r1, o1, n * sizeof(Fq), hipMemcpyDeviceToHost));
  CK(hipMemcpy(r2, o2, n * sizeof(Fq), hipMemcpyDeviceToHost));
  int bad1 = 0, bad2 = 0;
  for (int i = 0; i < n; i++) {
    for (int l = 0; l < 8; l++) {
      if (r0[i].v[l] != r1[i].v[l]) { bad1++; break; }
    }
    for (int l = 0; l < 8; l++) {
      if (r0[i].v[l] != r2[i].v[l]) { bad2++; break; }
    }
  }
  // host reference for the first few
  int badh = 0;
  for (int i = 0; i < 256; i++) {
    Fq xh, yh;
    CK(hipMemcpy(&xh, x + i, sizeof(Fq), hipMemcpyDeviceToHost));
    CK(hipMemcpy(&yh, y + i, sizeof(Fq), hipMemcpyDeviceToHost));
    Fq z = xh * yh;
    for (int l = 0; l < 8; l++) if (z.v[l] != r0[i].v[l]) { badh++; break; }
  }
  printf("{\"check\": {\"fips_vs_cios_mismatch\": %d, \"fips2_vs_cios_mismatch\": %d, \"cios_vs_host_mismatch\": %d}}\n", bad1, bad2, badh);
  run<0>("cios_c", io);
  run<1>("fips_asm", io);
  run<2>("fips_asm_dual", io);
  return (bad1 || bad2 || badh) ? 1 : 0;
}
