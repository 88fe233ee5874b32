// 9 x 29-bit-limb Montgomery arithmetic (R = 2^261) for the device hot loops.
//
// Why: with 29-bit limbs every column of a 254-bit product (<= 9 a*b plus
// 9 m*p partial products, each < 2^58) stays below 2^63, so each partial
// product is ONE v_mad_u64_u32 into a 64-bit accumulator — no carry-out, no
// v_addc, no VCC hazard nops.  Measured on MI355X (micro/fp29_bench.hip):
// 1.59e11 mul/s and 383 ns dependent latency, vs 1.18e11 and 789 ns for the
// 8 x 32-bit FIPS multiply in field.h.
//
// Values are plain integers in limb form; the Montgomery scale is bookkept by
// the caller (mul29(x, y) = x * y * 2^-261 mod p, output < 2p).  HBM keeps
// the 8 x 32-bit (arkworks) layout; conversion is re-limbing only.
//
// Limb invariants (documented per function):
//   normalized        every limb < 2^29
//   almost-normalized every limb < 2^29 + 8 (one parallel carry pass)
//   lazy              limbs < 2^31 (sums/differences of normalized values)
// mul29 needs one operand almost-normalized and the other at most lazy, and
// values below ~8p; then every column sum is < 2^64 and the output < 2p,
// normalized.
#pragma once
#include "field.h"

namespace qg {

static constexpr uint32_t M29 = (1u << 29) - 1;

struct L9 {
  uint32_t v[9];
};

constexpr L9 l9_from_words(const uint32_t (&w)[8]) {
  L9 r{};
  for (int i = 0; i < 9; i++) {
    const int lo = 29 * i, wi = lo / 32, s = lo % 32;
    uint64_t x = w[wi];
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << 32;
    r.v[i] = (uint32_t)(x >> s) & M29;
  }
  return r;
}

constexpr L9 l9_mul_small(const L9& a, uint32_t k) {
  L9 r{};
  uint64_t c = 0;
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)a.v[i] * k + c;
    r.v[i] = i < 8 ? (uint32_t)(t & M29) : (uint32_t)t;
    c = t >> 29;
  }
  return r;
}

// kp in a redundant form whose limbs 0..7 are >= 2^29 - 1 (+ kp's own limb):
// k - b has no negative limb for almost-normalized b.
constexpr L9 l9_redundant(const L9& kp) {
  L9 r{};
  r.v[0] = kp.v[0] + (1u << 29);
  for (int i = 1; i < 8; i++) r.v[i] = kp.v[i] + (1u << 29) - 1;
  r.v[8] = kp.v[8] - 1;
  return r;
}

constexpr uint32_t l9_inv29(uint32_t p0) {
  uint32_t x = p0;  // p0 * x == 1 mod 8 for odd p0
  for (int i = 0; i < 5; i++) x = x * (2u - p0 * x);
  return (0u - x) & M29;  // -p^-1 mod 2^29
}

constexpr bool l9_geq(const L9& a, const L9& b) {
  for (int i = 8; i >= 0; i--)
    if (a.v[i] != b.v[i]) return a.v[i] > b.v[i];
  return true;
}

constexpr L9 l9_sub(const L9& a, const L9& b) {
  L9 r{};
  uint32_t br = 0;
  for (int i = 0; i < 9; i++) {
    const uint32_t t = a.v[i] - b.v[i] - br;
    br = t >> 31;
    r.v[i] = i < 8 ? (t & M29) : t;
  }
  return r;
}

// 2^k mod p (plain integer), normalized limbs
constexpr L9 l9_pow2_mod(const L9& p, uint32_t k) {
  L9 x{};
  x.v[0] = 1;
  for (uint32_t j = 0; j < k; j++) {
    x = l9_mul_small(x, 2);
    if (l9_geq(x, p)) x = l9_sub(x, p);
  }
  return x;
}

struct L9x8 {
  L9 k[8];
};

constexpr L9x8 l9_multiples(const L9& p) {
  L9x8 r{};
  for (uint32_t k = 0; k < 8; k++) r.k[k] = l9_mul_small(p, k);
  return r;
}

struct L9x20 {
  L9 k[20];
};

constexpr L9x20 l9_multiples20(const L9& p) {
  L9x20 r{};
  for (uint32_t k = 0; k < 20; k++) r.k[k] = l9_mul_small(p, k);
  return r;
}

template <class C>
struct F29P {
  static constexpr L9 P = l9_from_words(C::P);
  static constexpr L9 P2 = l9_mul_small(P, 2);
  static constexpr L9 P4 = l9_mul_small(P, 4);
  static constexpr L9 P8 = l9_mul_small(P, 8);
  static constexpr L9 K4 = l9_redundant(l9_mul_small(P, 4));
  // 2p redundant: a + 2p - b for b < 2p (normalized) is exact in uint32 limb
  // arithmetic even when the top limb wraps (the value is >= 0, so the carry
  // into the top limb restores it in normfull29)
  static constexpr L9 K2 = l9_redundant(l9_mul_small(P, 2));
  static constexpr uint32_t INV = l9_inv29(C::P[0]);
  static constexpr L9 ONE = l9_pow2_mod(P, 261);     // 1 in the R = 2^261 domain
  static constexpr L9 TO261 = l9_pow2_mod(P, 266);   // mul29(x 2^256, .) = x 2^261
  static constexpr L9 TO256 = l9_pow2_mod(P, 256);   // mul29(x 2^261, .) = x 2^256
  static constexpr L9x8 KP = l9_multiples(P);        // 0, p, ..., 7p
  static constexpr L9x20 KP20 = l9_multiples20(P);   // 0, p, ..., 19p
  static constexpr L9 K9 = l9_redundant(l9_mul_small(P, 9));    // subtrahends < 8p
  static constexpr L9 K17 = l9_redundant(l9_mul_small(P, 17));  // subtrahends < 16p
};

template <class C>
struct F29 {
  uint32_t l[9];
  QG_HD static F29 zero() {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = 0;
    return r;
  }
  QG_HD static F29 from_l9(const L9& x) {
    F29 r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = x.v[i];
    return r;
  }
};

// 8 x 32 words (value < 2^256) -> normalized limbs, same integer
template <class C>
QG_HD F29<C> to29(const Fp<C>& x) {
  F29<C> r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int lo = 29 * i, w = lo >> 5, s = lo & 31;
    uint64_t v = x.v[w];
    if (w + 1 < 8) v |= (uint64_t)x.v[w + 1] << 32;
    r.l[i] = (uint32_t)(v >> s) & M29;
  }
  return r;
}

// normalized limbs (value < 2^256) -> 8 x 32 words, same integer
template <class C>
QG_HD Fp<C> from29(const F29<C>& a) {
  Fp<C> r;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    const int lo = 32 * w, i = lo / 29, s = lo % 29;
    uint64_t v = (uint64_t)a.l[i] >> s;
    if (i + 1 < 9) v |= (uint64_t)a.l[i + 1] << (29 - s);
    if (i + 2 < 9) v |= (uint64_t)a.l[i + 2] << (58 - s);
    r.v[w] = (uint32_t)v;
  }
  return r;
}

// Montgomery product x * y * 2^-261 mod p (< 2p, normalized); see header for
// the operand conditions.
template <class C>
QG_HD F29<C> mul29(const F29<C>& a, const F29<C>& b) {
  uint32_t m[9];
  F29<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      acc += (uint64_t)m[j] * F29P<C>::P.v[k - j];
    }
    acc += (uint64_t)a.l[k] * b.l[0];
    m[k] = ((uint32_t)acc * F29P<C>::INV) & M29;
    acc += (uint64_t)m[k] * F29P<C>::P.v[0];
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      acc += (uint64_t)m[j] * F29P<C>::P.v[k - j];
    }
    r.l[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// Montgomery square a^2 * 2^-261 (< 2p): cross products once with 2a
// (45 + 81 partial products instead of 81 + 81); a almost-normalized.
template <class C>
QG_HD F29<C> sqr29(const F29<C>& a) {
  uint32_t a2[9], m[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.l[i] << 1;
  F29<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) acc += (uint64_t)a2[i] * a.l[k - i];
    if ((k & 1) == 0) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
    if (k < 9) {
#pragma unroll
      for (int j = 0; j < k; j++) acc += (uint64_t)m[j] * F29P<C>::P.v[k - j];
      m[k] = ((uint32_t)acc * F29P<C>::INV) & M29;
      acc += (uint64_t)m[k] * F29P<C>::P.v[0];
    } else {
#pragma unroll
      for (int j = k - 8; j < 9; j++) acc += (uint64_t)m[j] * F29P<C>::P.v[k - j];
      r.l[k - 9] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// (a b - c d) 2^-261 + 4p (mod p), one Montgomery reduction for both
// products; signed column accumulation.  a, b, c, d almost-normalized,
// c d < 4p 2^261.  Output normalized, value < a b 2^-261 + 5p.
template <class C>
QG_HD F29<C> mulsub29(const F29<C>& a, const F29<C>& b, const F29<C>& c, const F29<C>& d) {
  int32_t nd[9];
  uint32_t m[9];
#pragma unroll
  for (int i = 0; i < 9; i++) nd[i] = -(int32_t)d.l[i];
  F29<C> r;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int j = (k > 8 ? k - 8 : 0); j <= (k < 8 ? k : 8); j++) {
      acc += (int64_t)((uint64_t)a.l[j] * b.l[k - j]);
      // both factors as int32 (c's limbs < 2^30): one v_mad_i64_i32, not an
      // unsigned product plus a sign correction
      acc += (int64_t)(int32_t)c.l[j] * (int64_t)nd[k - j];
    }
    if (k < 9) {
#pragma unroll
      for (int j = 0; j < k; j++) acc += (int64_t)((uint64_t)m[j] * F29P<C>::P.v[k - j]);
      m[k] = ((uint32_t)acc * F29P<C>::INV) & M29;
      acc += (int64_t)((uint64_t)m[k] * F29P<C>::P.v[0]);
    } else {
#pragma unroll
      for (int j = k - 8; j < 9; j++) acc += (int64_t)((uint64_t)m[j] * F29P<C>::P.v[k - j]);
      acc += F29P<C>::P4.v[k - 9];
      r.l[k - 9] = (uint32_t)acc & M29;
    }
    acc >>= 29;  // arithmetic
  }
  r.l[8] = (uint32_t)(acc + F29P<C>::P4.v[8]);
  return r;
}

#if defined(__HIP_DEVICE_COMPILE__)
// ---- throughput variants (device only) -------------------------------------
// Same arithmetic as mul29 / sqr29 / mulsub29, but every column is ONE
// accumulation chain of v_mad_u64_u32 (inline asm: the compiler cannot
// re-associate a column into two chains merged by v_lshl_add_u64), and the
// modulus limbs are SGPR operands.  ~17 fewer VALU instructions per multiply
// (+8 % multiplies/s in micro/fp29_bench.hip) at a longer dependent latency
// (616 vs 383 ns): for kernels with many independent multiplies in flight
// (the MSM bucket accumulation), not for latency-bound chains.
// a * b + c with the result made opaque to the optimizer by an empty asm
// statement (no instruction is emitted): the column stays one chain.  The
// product itself is the compiler's v_mad_u64_u32.
__device__ __forceinline__ uint64_t mad_vv(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r = (uint64_t)a * b + c;
#ifndef QG_MAD_PLAIN
  asm("" : "+v"(r));
#endif
  return r;
}
__device__ __forceinline__ uint64_t mad_vs(uint32_t a, uint32_t b, uint64_t c) {
  return mad_vv(a, b, c);
}
__device__ __forceinline__ int64_t mad_i_vv(int32_t a, int32_t b, int64_t c) {
  int64_t r = (int64_t)a * b + c;
#ifndef QG_MAD_PLAIN
  asm("" : "+v"(r));
#endif
  return r;
}
__device__ __forceinline__ int64_t mad_u_signed(uint32_t a, uint32_t b, int64_t c) {
  return (int64_t)mad_vv(a, b, (uint64_t)c);  // two's complement: same bits
}
__device__ __forceinline__ int64_t mad_s_signed(uint32_t a, uint32_t b, int64_t c) {
  return (int64_t)mad_vs(a, b, (uint64_t)c);
}

template <class C>
__device__ __forceinline__ F29<C> mul29t(const F29<C>& a, const F29<C>& b) {
  uint32_t m[9];
  F29<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      acc = mad_vv(a.l[j], b.l[k - j], acc);
      acc = mad_vs(m[j], F29P<C>::P.v[k - j], acc);
    }
    acc = mad_vv(a.l[k], b.l[0], acc);
    m[k] = ((uint32_t)acc * F29P<C>::INV) & M29;
    acc = mad_vs(m[k], F29P<C>::P.v[0], acc);
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
      acc = mad_vv(a.l[j], b.l[k - j], acc);
      acc = mad_vs(m[j], F29P<C>::P.v[k - j], acc);
    }
    r.l[k - 9] = (uint32_t)acc & M29;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

template <class C>
__device__ __forceinline__ F29<C> sqr29t(const F29<C>& a) {
  uint32_t a2[9], m[9];
#pragma unroll
  for (int i = 0; i < 9; i++) a2[i] = a.l[i] << 1;
  F29<C> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) acc = mad_vv(a2[i], a.l[k - i], acc);
    if ((k & 1) == 0) acc = mad_vv(a.l[k / 2], a.l[k / 2], acc);
    if (k < 9) {
#pragma unroll
      for (int j = 0; j < k; j++) acc = mad_vs(m[j], F29P<C>::P.v[k - j], acc);
      m[k] = ((uint32_t)acc * F29P<C>::INV) & M29;
      acc = mad_vs(m[k], F29P<C>::P.v[0], acc);
    } else {
#pragma unroll
      for (int j = k - 8; j < 9; j++) acc = mad_vs(m[j], F29P<C>::P.v[k - j], acc);
      r.l[k - 9] = (uint32_t)acc & M29;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// Two independent products with their column chains interleaved mad by mad:
// no v_mad_u64_u32 result is read by the next instruction, so the hazard
// s_nop gfx950 places after every dependent mad of a single chain goes away
// (micro/pair_bench.hip: +2.5 % multiplies/s at full occupancy).  Same
// arithmetic and operand conditions as mul29t / sqr29t.
template <class C>
__device__ __forceinline__ void mul29t2(const F29<C>& a, const F29<C>& b, const F29<C>& c,
                                        const F29<C>& d, F29<C>& r1, F29<C>& r2) {
  uint32_t m[9], n[9];
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      x = mad_vv(a.l[j], b.l[k - j], x);
      y = mad_vv(c.l[j], d.l[k - j], y);
      x = mad_vs(m[j], F29P<C>::P.v[k - j], x);
      y = mad_vs(n[j], F29P<C>::P.v[k - j], y);
    }
    x = mad_vv(a.l[k], b.l[0], x);
    y = mad_vv(c.l[k], d.l[0], y);
    m[k] = ((uint32_t)x * F29P<C>::INV) & M29;
    n[k] = ((uint32_t)y * F29P<C>::INV) & M29;
    x = mad_vs(m[k], F29P<C>::P.v[0], x);
    y = mad_vs(n[k], F29P<C>::P.v[0], y);
    x >>= 29;
    y >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
      x = mad_vv(a.l[j], b.l[k - j], x);
      y = mad_vv(c.l[j], d.l[k - j], y);
      x = mad_vs(m[j], F29P<C>::P.v[k - j], x);
      y = mad_vs(n[j], F29P<C>::P.v[k - j], y);
    }
    r1.l[k - 9] = (uint32_t)x & M29;
    r2.l[k - 9] = (uint32_t)y & M29;
    x >>= 29;
    y >>= 29;
  }
  r1.l[8] = (uint32_t)x;
  r2.l[8] = (uint32_t)y;
}

template <class C>
__device__ __forceinline__ void sqr29t2(const F29<C>& a, const F29<C>& c, F29<C>& r1,
                                        F29<C>& r2) {
  uint32_t a2[9], c2[9], m[9], n[9];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    a2[i] = a.l[i] << 1;
    c2[i] = c.l[i] << 1;
  }
  uint64_t x = 0, y = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = (k > 8 ? k - 8 : 0); 2 * i < k; i++) {
      x = mad_vv(a2[i], a.l[k - i], x);
      y = mad_vv(c2[i], c.l[k - i], y);
    }
    if ((k & 1) == 0) {
      x = mad_vv(a.l[k / 2], a.l[k / 2], x);
      y = mad_vv(c.l[k / 2], c.l[k / 2], y);
    }
    if (k < 9) {
#pragma unroll
      for (int j = 0; j < k; j++) {
        x = mad_vs(m[j], F29P<C>::P.v[k - j], x);
        y = mad_vs(n[j], F29P<C>::P.v[k - j], y);
      }
      m[k] = ((uint32_t)x * F29P<C>::INV) & M29;
      n[k] = ((uint32_t)y * F29P<C>::INV) & M29;
      x = mad_vs(m[k], F29P<C>::P.v[0], x);
      y = mad_vs(n[k], F29P<C>::P.v[0], y);
    } else {
#pragma unroll
      for (int j = k - 8; j < 9; j++) {
        x = mad_vs(m[j], F29P<C>::P.v[k - j], x);
        y = mad_vs(n[j], F29P<C>::P.v[k - j], y);
      }
      r1.l[k - 9] = (uint32_t)x & M29;
      r2.l[k - 9] = (uint32_t)y & M29;
    }
    x >>= 29;
    y >>= 29;
  }
  r1.l[8] = (uint32_t)x;
  r2.l[8] = (uint32_t)y;
}

// N independent products r[n] = a[n] b[n] 2^-261 with their column chains
// interleaved mad by mad (mul29t2 generalised): consecutive mads belong to
// different chains, so no hazard s_nop, and N chains are in flight for the
// wave.  Same arithmetic and operand conditions as mul29t.  r may alias a.
template <class C, int N>
__device__ __forceinline__ void mul29tn(const F29<C> (&a)[N], const F29<C> (&b)[N],
                                        F29<C> (&r)[N]) {
  uint32_t m[N][9];
  uint64_t x[N];
#pragma unroll
  for (int n = 0; n < N; n++) x[n] = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
#pragma unroll
      for (int n = 0; n < N; n++) x[n] = mad_vv(a[n].l[j], b[n].l[k - j], x[n]);
#pragma unroll
      for (int n = 0; n < N; n++) x[n] = mad_vs(m[n][j], F29P<C>::P.v[k - j], x[n]);
    }
#pragma unroll
    for (int n = 0; n < N; n++) x[n] = mad_vv(a[n].l[k], b[n].l[0], x[n]);
#pragma unroll
    for (int n = 0; n < N; n++) m[n][k] = ((uint32_t)x[n] * F29P<C>::INV) & M29;
#pragma unroll
    for (int n = 0; n < N; n++) x[n] = mad_vs(m[n][k], F29P<C>::P.v[0], x[n]) >> 29;
  }
  uint32_t out[N][9];
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int j = k - 8; j < 9; j++) {
#pragma unroll
      for (int n = 0; n < N; n++) x[n] = mad_vv(a[n].l[j], b[n].l[k - j], x[n]);
#pragma unroll
      for (int n = 0; n < N; n++) x[n] = mad_vs(m[n][j], F29P<C>::P.v[k - j], x[n]);
    }
#pragma unroll
    for (int n = 0; n < N; n++) {
      out[n][k - 9] = (uint32_t)x[n] & M29;
      x[n] >>= 29;
    }
  }
#pragma unroll
  for (int n = 0; n < N; n++) {
#pragma unroll
    for (int i = 0; i < 8; i++) r[n].l[i] = out[n][i];
    r[n].l[8] = (uint32_t)x[n];
  }
}

// mulsub29 with one signed chain per column
template <class C>
__device__ __forceinline__ F29<C> mulsub29t(const F29<C>& a, const F29<C>& b, const F29<C>& c,
                                            const F29<C>& d) {
  int32_t nd[9];
  uint32_t m[9];
#pragma unroll
  for (int i = 0; i < 9; i++) nd[i] = -(int32_t)d.l[i];
  F29<C> r;
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int j = (k > 8 ? k - 8 : 0); j <= (k < 8 ? k : 8); j++) {
      acc = mad_u_signed(a.l[j], b.l[k - j], acc);
      acc = mad_i_vv((int32_t)c.l[j], nd[k - j], acc);
    }
    if (k < 9) {
#pragma unroll
      for (int j = 0; j < k; j++) acc = mad_s_signed(m[j], F29P<C>::P.v[k - j], acc);
      m[k] = ((uint32_t)acc * F29P<C>::INV) & M29;
      acc = mad_s_signed(m[k], F29P<C>::P.v[0], acc);
    } else {
#pragma unroll
      for (int j = k - 8; j < 9; j++) acc = mad_s_signed(m[j], F29P<C>::P.v[k - j], acc);
      acc += F29P<C>::P4.v[k - 9];
      r.l[k - 9] = (uint32_t)acc & M29;
    }
    acc >>= 29;  // arithmetic
  }
  r.l[8] = (uint32_t)(acc + F29P<C>::P4.v[8]);
  return r;
}
#elif defined(__HIP__)
// host pass: declarations only (device code, never called from the host)
template <class C, int N>
__device__ void mul29tn(const F29<C> (&a)[N], const F29<C> (&b)[N], F29<C> (&r)[N]);
template <class C>
__device__ F29<C> mul29t(const F29<C>& a, const F29<C>& b);
template <class C>
__device__ F29<C> sqr29t(const F29<C>& a);
template <class C>
__device__ F29<C> mulsub29t(const F29<C>& a, const F29<C>& b, const F29<C>& c, const F29<C>& d);
template <class C>
__device__ void mul29t2(const F29<C>& a, const F29<C>& b, const F29<C>& c, const F29<C>& d,
                        F29<C>& r1, F29<C>& r2);
template <class C>
__device__ void sqr29t2(const F29<C>& a, const F29<C>& c, F29<C>& r1, F29<C>& r2);
#endif

// limb-wise sum (lazy)
template <class C>
QG_HD F29<C> add29(const F29<C>& a, const F29<C>& b) {
  F29<C> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}

// a + 4p - b (lazy, value a + 4p - b > 0); b almost-normalized, value < 4p
template <class C>
QG_HD F29<C> sub29(const F29<C>& a, const F29<C>& b) {
  F29<C> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + (F29P<C>::K4.v[i] - b.l[i]);
  return r;
}

// a + k - b with a redundant multiple k of p (subtrahend value below k - p)
template <class C>
QG_HD F29<C> subk29(const F29<C>& a, const F29<C>& b, const L9& k) {
  F29<C> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + (k.v[i] - b.l[i]);
  return r;
}

// one parallel carry pass: limbs < 2^32 -> almost-normalized (< 2^29 + 8)
template <class C>
QG_HD F29<C> norm29(const F29<C>& a) {
  F29<C> r;
  r.l[0] = a.l[0] & M29;
#pragma unroll
  for (int i = 1; i < 9; i++) r.l[i] = (a.l[i] & M29) + (a.l[i - 1] >> 29);
  r.l[8] = a.l[8] + (a.l[7] >> 29);
  return r;
}

// full carry propagation -> normalized (top limb takes the excess)
template <class C>
QG_HD F29<C> normfull29(const F29<C>& a) {
  F29<C> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t t = a.l[i] + c;
    r.l[i] = t & M29;
    c = t >> 29;
  }
  r.l[8] = a.l[8] + c;
  return r;
}

// normalized a (value < 2^261) -> a - k if a >= k else a   (k normalized)
template <class C>
QG_HD F29<C> condsub29(const F29<C>& a, const L9& k) {
  F29<C> d;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t t = a.l[i] - k.v[i] - br;
    br = t >> 31;
    d.l[i] = t & M29;
  }
  // br == 1: a < k, keep a
  F29<C> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = br ? a.l[i] : d.l[i];
  return r;
}

// lazy value < 4p -> normalized, < 2p
template <class C>
QG_HD F29<C> red2p29(const F29<C>& a) {
  return condsub29<C>(normfull29<C>(a), F29P<C>::P2);
}

// lazy value < 16p -> normalized, < 2p
template <class C>
QG_HD F29<C> red16p29(const F29<C>& a) {
  F29<C> x = condsub29<C>(normfull29<C>(a), F29P<C>::P8);
  x = condsub29<C>(x, F29P<C>::P4);
  return condsub29<C>(x, F29P<C>::P2);
}

// lazy value < 6p -> normalized, < 2p
template <class C>
QG_HD F29<C> red6p29(const F29<C>& a) {
  return condsub29<C>(condsub29<C>(normfull29<C>(a), F29P<C>::P4), F29P<C>::P2);
}

// normalized value < 8p: is it 0 mod p?  (low-limb filter, then exact check)
template <class C>
QG_HD bool is_zero_mod29(const F29<C>& a) {
  bool z = false;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    if (a.l[0] == F29P<C>::KP.k[k].v[0]) {
      bool eq = true;
#pragma unroll
      for (int i = 1; i < 9; i++) eq = eq && a.l[i] == F29P<C>::KP.k[k].v[i];
      z = z || eq;
    }
  }
  return z;
}

// normalized value < K p (K <= 20): is it 0 mod p?  a = k p forces
// k == l0 p^-1 (mod 2^29), so one multiply rejects every nonzero residue but a
// K / 2^29 fraction, and only those run the exact limb comparison with k p
// (the compare loops of is_zero_mod29 cost ~100 VALU + exec-mask SALU per test).
template <class C, int K>
QG_HD bool is_zero_mod29_fast(const F29<C>& a) {
  const uint32_t k = (0u - a.l[0] * F29P<C>::INV) & M29;
  if (k >= (uint32_t)K) return false;
  uint64_t c = 0;
  bool eq = true;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t t = (uint64_t)F29P<C>::P.v[i] * k + c;
    const uint32_t limb = i < 8 ? (uint32_t)(t & M29) : (uint32_t)t;
    c = t >> 29;
    eq = eq && limb == a.l[i];
  }
  return eq;
}

// normalized value < 20p: is it 0 mod p?
template <class C>
QG_HD bool is_zero_mod29_20(const F29<C>& a) {
  bool z = false;
#pragma unroll
  for (int k = 0; k < 20; k++) {
    if (a.l[0] == F29P<C>::KP20.k[k].v[0]) {
      bool eq = true;
#pragma unroll
      for (int i = 1; i < 9; i++) eq = eq && a.l[i] == F29P<C>::KP20.k[k].v[i];
      z = z || eq;
    }
  }
  return z;
}

// a^(p-2) in the R = 2^261 domain (a in that domain, normalized < 2p)
template <class C>
QG_HD F29<C> inv29(const F29<C>& a) {
  uint32_t e[8];
  uint32_t br = 0;
  e[0] = subb32(C::P[0], 2u, 0, &br);
  for (int i = 1; i < 8; i++) e[i] = subb32(C::P[i], 0u, br, &br);
  F29<C> r = F29<C>::from_l9(F29P<C>::ONE);
  for (int i = 7; i >= 0; i--) {
    for (int bit = 31; bit >= 0; bit--) {
      r = mul29(r, r);
      if ((e[i] >> bit) & 1u) r = mul29(r, a);
    }
  }
  return r;
}

// normalized value < 2p -> canonical (< p)
template <class C>
QG_HD F29<C> canon29(const F29<C>& a) {
  return condsub29<C>(a, F29P<C>::P);
}

template <class C>
QG_HD bool is_zero29(const F29<C>& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) acc |= a.l[i];
  return acc == 0;
}

#if defined(__HIPCC__) || defined(__HIP__)
template <class C>
QG_DEV F29<C> shfl_xor29(const F29<C>& a, int m) {
  F29<C> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = __shfl_xor(a.l[i], m, 64);
  return r;
}
#endif

// host: 2^k mod p as a plain integer (8 x 32 words)
template <class C>
inline Fp<C> pow2_mod_plain(uint32_t k) {
  Fp<C> x = Fp<C>::zero();
  x.v[0] = 1;
  for (uint32_t i = 0; i < k; i++) x = x + x;  // modular doubling of a plain integer < p
  return x;
}

}  // namespace qg
