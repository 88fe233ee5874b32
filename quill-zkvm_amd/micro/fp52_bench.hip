// FP64-FMA Montgomery multiply over BN254 Fq in 5 x 52-bit limbs (R = 2^260)
// against the in-tree 9 x 29-bit mul29t (R = 2^261): multiplies/s over the
// whole chip, same harness shape as pair_bench.hip (4 independent chains per
// thread, 256 x 32 blocks).  VERDICT r2 item 5: port only if >= 1.25x.
//
// Partial products are split exactly with two FMAs (Dekker-style, the
// "DPF" layout of Emmart & Weems): for integers x, y < 2^52
//   hc = fma(x, y, 2^104)          = 2^104 + hi,  hi = round(xy / 2^52) 2^52
//   lo = fma(x, y, -(hc - 2^104))  = xy - hi,     |lo| <= 2^51
// The raw bit pattern of hc minus that of 2^104 is hi / 2^52 (the exponent is
// fixed inside [2^104, 2^105)); lo + 1.5 2^52 lies in [2^52, 2^53), whose raw
// bits minus those of 1.5 2^52 are lo.  Columns accumulate those integers in
// int64 (<= 20 terms of < 2^53: no overflow).  Montgomery reduction per limb:
// m = (col * p') mod 2^52, then the same split for m * p_j.
// Correctness: mont52(a, b) = a b 2^-260 = 2 mul29(a, b) mod p, checked on
// the device for every thread of a check grid (canonical 8 x 32 words).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../csrc/field29.h"
using namespace qg;
using Q = F29<FqP>;

struct P52 {
  double p[5];      // p in 52-bit limbs
  uint64_t pinv;    // -p^-1 mod 2^52
};

static constexpr double C104 = 20282409603651670423947251286016.0;  // 2^104
static constexpr double B52 = 6755399441055744.0;                    // 1.5 * 2^52
static constexpr uint64_t M52 = (1ull << 52) - 1;

__device__ __forceinline__ int64_t bits(double x) { return __double_as_longlong(x); }

// acc[k] += lo, acc[k+1] += hi of x * y (raw-bit accumulation, offsets removed
// later; unsigned: the raw patterns wrap, the true column values do not)
__device__ __forceinline__ void split_acc(double x, double y, uint64_t& lo_acc, uint64_t& hi_acc) {
  const double hc = __fma_rn(x, y, C104);
  const double hi = hc - C104;
  const double lo = __fma_rn(x, y, -hi) + B52;
  hi_acc += (uint64_t)bits(hc);
  lo_acc += (uint64_t)bits(lo);
}

struct F52 {
  double l[5];
};

__device__ __forceinline__ F52 mont52(const F52& a, const F52& b, const P52& P) {
  const uint64_t HB = (uint64_t)bits(C104), LB = (uint64_t)bits(B52);
  uint64_t acc[10];
#pragma unroll
  for (int k = 0; k < 10; k++) acc[k] = 0;
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int j = 0; j < 5; j++) split_acc(a.l[i], b.l[j], acc[i + j], acc[i + j + 1]);
  // remove the offsets: column k got n_lo(k) LB and n_hi(k) HB (compile-time counts)
#pragma unroll
  for (int k = 0; k < 10; k++) {
    const int nlo = k <= 8 ? (k < 5 ? k + 1 : 9 - k) : 0;
    const int nhi = k >= 1 ? (k <= 5 ? k : 10 - k) : 0;
    acc[k] -= (uint64_t)nlo * LB + (uint64_t)nhi * HB;
  }
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const uint64_t m = (acc[i] * P.pinv) & M52;
    const double md = (double)m;
#pragma unroll
    for (int j = 0; j < 5; j++) {
      uint64_t l = 0, h = 0;
      split_acc(md, P.p[j], l, h);
      acc[i + j] += l - LB;
      acc[i + j + 1] += h - HB;
    }
    acc[i + 1] += (uint64_t)((int64_t)acc[i] >> 52);  // acc[i] == 0 mod 2^52 now
  }
  F52 r;
#pragma unroll
  for (int k = 5; k < 9; k++) {
    const int64_t v = (int64_t)acc[k];
    r.l[k - 5] = (double)(v & (int64_t)M52);
    acc[k + 1] += (uint64_t)(v >> 52);
  }
  // top limb: everything from bit 208 up (the result is < 2p < 2^255)
  r.l[4] = (double)(int64_t)acc[9];
  return r;
}

__device__ F52 from_words(const uint32_t* w) {  // 8 x 32 LE -> 5 x 52
  uint64_t x[4];
  for (int i = 0; i < 4; i++) x[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
  F52 r;
  r.l[0] = (double)(x[0] & M52);
  r.l[1] = (double)(((x[0] >> 52) | (x[1] << 12)) & M52);
  r.l[2] = (double)(((x[1] >> 40) | (x[2] << 24)) & M52);
  r.l[3] = (double)(((x[2] >> 28) | (x[3] << 36)) & M52);
  r.l[4] = (double)(x[3] >> 16);
  return r;
}

__device__ void to_words(const F52& a, uint32_t* w) {  // (a < 2^256) -> 8 x 32 LE
  unsigned __int128 acc = 0;
  uint64_t x[4] = {0, 0, 0, 0};
  int bit = 0, word = 0;
  for (int i = 0; i < 5; i++) {
    acc |= (unsigned __int128)(uint64_t)a.l[i] << bit;
    bit += 52;
    while (bit >= 64 && word < 4) {
      x[word++] = (uint64_t)acc;
      acc >>= 64;
      bit -= 64;
    }
  }
  if (word < 4) x[word] = (uint64_t)acc;
  for (int i = 0; i < 4; i++) {
    w[2 * i] = (uint32_t)x[i];
    w[2 * i + 1] = (uint32_t)(x[i] >> 32);
  }
}

__device__ Q load29(const Fq* io, size_t i) { return to29(io[i & 1023]); }
__device__ F52 load52(const Fq* io, size_t i) { return from_words(io[i & 1023].v); }

template <int V>
__global__ void __launch_bounds__(256) k_tp(Fq* io, int iters, P52 P) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s = 0;
  if constexpr (V == 0) {
    Q a[4], b = load29(io, i);
    for (int k = 0; k < 4; k++) a[k] = load29(io, i + k + 1);
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = mul29t(a[k], b);
    }
    for (int k = 0; k < 4; k++)
      for (int l = 0; l < 9; l++) s ^= a[k].l[l] * (2 * l + 1);
  } else {
    F52 a[4], b = load52(io, i);
    for (int k = 0; k < 4; k++) a[k] = load52(io, i + k + 1);
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int k = 0; k < 4; k++) a[k] = mont52(a[k], b, P);
    }
    for (int k = 0; k < 4; k++)
      for (int l = 0; l < 5; l++) s ^= (uint32_t)(uint64_t)a[k].l[l] * (2 * l + 1);
  }
  if (s == 0x12345678u) io[i & 1023].v[0] = s;
}

// canonical 8 x 32 words of a value < 4p
__device__ void canon_words(uint32_t* t) {
  for (int r = 0; r < 3; r++) reduce_once<FqP>(t);
}

__global__ void k_check(const Fq* io, uint32_t* out, int iters, P52 P) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  // chain of `iters` multiplies in both forms; x52 tracks 2^(iters) x29
  // because each mont52 step is 2 x mul29: compare x52 with 2^iters x29 mod p
  Q x = load29(io, i), b = load29(io, i + 3);
  F52 u = load52(io, i), v = load52(io, i + 3);
  for (int it = 0; it < iters; it++) {
    x = mul29t(x, b);
    u = mont52(u, v, P);
  }
  // scale x by 2^iters: x29 -> words, double iters times mod p
  Fq xw = from29(x);
  uint32_t t[8];
  for (int k = 0; k < 8; k++) t[k] = xw.v[k];
  canon_words(t);
  for (int it = 0; it < iters; it++) {
    uint32_t c = 0;
    for (int k = 0; k < 8; k++) {
      const uint32_t nv = (t[k] << 1) | c;
      c = t[k] >> 31;
      t[k] = nv;
    }
    canon_words(t);
  }
  uint32_t w[8];
  to_words(u, w);
  canon_words(w);
  uint32_t bad = 0;
  for (int k = 0; k < 8; k++) bad |= t[k] ^ w[k];
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
static double run(const char* name, Fq* io, const P52& P) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const unsigned blocks = 256 * 32;
  const int iters = 256;
  k_tp<V><<<blocks, 256>>>(io, 8, P);
  CK(hipEventRecord(a));
  k_tp<V><<<blocks, 256>>>(io, iters, P);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double r = (double)blocks * 256 * 4 * iters / (ms * 1e-3);
  printf("{\"variant\": \"%s\", \"mul_per_s\": %.4g, \"ms\": %.3f}\n", name, r, ms);
  return r;
}

int main() {
  // p = BN254 Fq, little-endian 64-bit limbs
  const uint64_t p64[4] = {0x3C208C16D87CFD47ull, 0x97816A916871CA8Dull, 0xB85045B68181585Dull,
                           0x30644E72E131A029ull};
  P52 P;
  P.p[0] = (double)(p64[0] & M52);
  P.p[1] = (double)(((p64[0] >> 52) | (p64[1] << 12)) & M52);
  P.p[2] = (double)(((p64[1] >> 40) | (p64[2] << 24)) & M52);
  P.p[3] = (double)(((p64[2] >> 28) | (p64[3] << 36)) & M52);
  P.p[4] = (double)(p64[3] >> 16);
  // -p^-1 mod 2^64 by Newton, then mod 2^52
  uint64_t inv = 1;
  for (int k = 0; k < 7; k++) inv *= 2 - p64[0] * inv;
  P.pinv = (0 - inv) & M52;
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
    h[i].v[7] &= 0x1fffffffu;  // < 2^253 < p
  }
  CK(hipMemcpy(io, h, sizeof(h), hipMemcpyHostToDevice));
  k_check<<<64, 256>>>(io, bad, 40, P);
  uint32_t nb = 0;
  CK(hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost));
  printf("{\"check_mismatch_threads\": %u, \"checked_threads\": %d}\n", nb, 64 * 256);
  double r29 = 0, r52 = 0;
  for (int rep = 0; rep < 2; rep++) {
    r29 = run<0>("mul29t_x4", io, P);
    r52 = run<1>("mont52_fma_x4", io, P);
  }
  printf("{\"fp52_over_mul29t\": %.3f}\n", r52 / r29);
  return nb ? 1 : 0;
}
