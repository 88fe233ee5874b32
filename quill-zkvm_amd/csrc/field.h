// BN254 prime-field arithmetic for gfx950 (and the host side of the library).
//
// Elements are 8 x 32-bit little-endian limbs in Montgomery form with
// R = 2^256.  That is byte-for-byte arkworks' in-memory `Fp256(BigInt([u64;4]))`
// (ark-ff 0.5.0, Cargo.lock:56-57), so scalars cross the C-ABI with zero
// conversion.  Multiplication is CIOS with the "no final carry word"
// shortcut: both BN254 moduli have a top limb 0x30644e72 < 2^31 - 1, so the
// running value stays below 2q and fits 8 limbs.  Each 32x32+32+32 step maps
// to one v_mad_u64_u32 plus a carry add on CDNA4; there is no MFMA form of
// 256-bit modular products.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define QG_HD __host__ __device__ __forceinline__
#define QG_DEV __device__ __forceinline__
#else
#define QG_HD inline
#define QG_DEV inline
#endif

namespace qg {

struct FrP {
  static constexpr uint32_t P[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xefffffffu;  // -P^{-1} mod 2^32
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr uint32_t R3[8] = {0xb4bf0040u, 0x5e94d8e1u, 0x1cfbb6b8u, 0x2a489cbeu,
                                     0xa19fcfedu, 0x893cc664u, 0x7fcc657cu, 0x0cf8594bu};
  static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
};

struct FqP {
  static constexpr uint32_t P[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xe4866389u;
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr uint32_t R3[8] = {0xda1530dfu, 0xb1cd6dafu, 0xa7283db6u, 0x62f210e6u,
                                     0x0ada0afbu, 0xef7f0b0cu, 0x2d592544u, 0x20fd6e90u};
  static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
};

template <class C>
struct Fp {
  uint32_t v[8];

  QG_HD static Fp zero() {
    Fp r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  QG_HD static Fp one() {
    Fp r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = C::ONE[i];
    return r;
  }
  QG_HD static Fp from_raw(const uint32_t* p) {
    Fp r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = p[i];
    return r;
  }
  QG_HD bool is_zero() const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i];
    return acc == 0;
  }
  QG_HD bool operator==(const Fp& o) const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= (v[i] ^ o.v[i]);
    return acc == 0;
  }
  QG_HD bool operator!=(const Fp& o) const { return !(*this == o); }
};

using Fr = Fp<FrP>;
using Fq = Fp<FqP>;

// ---- limb helpers ---------------------------------------------------------
QG_HD uint32_t addc32(uint32_t a, uint32_t b, uint32_t cin, uint32_t* cout) {
  uint64_t s = (uint64_t)a + b + cin;
  *cout = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
QG_HD uint32_t subb32(uint32_t a, uint32_t b, uint32_t bin, uint32_t* bout) {
  uint64_t d = (uint64_t)a - b - bin;
  *bout = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

// r = t - P if t >= P else t   (t < 2P)
template <class C>
QG_HD void reduce_once(uint32_t t[8]) {
  uint32_t s[8], b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s[i] = subb32(t[i], C::P[i], b, &b);
  // b == 1 -> t < P, keep t
  uint32_t keep = 0u - b;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = (t[i] & keep) | (s[i] & ~keep);
}

template <class C>
QG_HD Fp<C> operator+(const Fp<C>& a, const Fp<C>& b) {
  Fp<C> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(a.v[i], b.v[i], c, &c);
  reduce_once<C>(r.v);
  return r;
}

template <class C>
QG_HD Fp<C> operator-(const Fp<C>& a, const Fp<C>& b) {
  Fp<C> r;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = subb32(a.v[i], b.v[i], br, &br);
  // if borrow, add P back
  uint32_t mask = 0u - br, c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = addc32(r.v[i], C::P[i] & mask, c, &c);
  return r;
}

template <class C>
QG_HD Fp<C> fneg(const Fp<C>& a) {
  return Fp<C>::zero() - a;
}

template <class C>
QG_HD Fp<C> fdbl(const Fp<C>& a) {
  return a + a;
}

#if defined(__HIP_DEVICE_COMPILE__)
// (acc:64, hi:32) += a * b  — one v_mad_u64_u32 with its carry-out in VCC
// folded into the third accumulator word by one v_addc.  hipcc does not emit
// the carry-out form itself (it rebuilds 64-bit addends with v_mov pairs).
__device__ __forceinline__ void mac96(uint64_t& acc, uint32_t& hi, uint32_t a, uint32_t b) {
  uint64_t r;
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %4\n\t"
      "v_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
      : "=&v"(r), "+v"(hi)
      : "v"(a), "v"(b), "v"(acc)
      : "vcc");
  acc = r;
}

// Montgomery product, FIPS (finely integrated product scanning): column k of
// a*b and m*P accumulate in a 96-bit register accumulator; m_k is formed from
// the column's low word.  2 instructions per 32x32 product; measured 1.25e11
// mul/s on MI355X vs 0.91e11 for the C CIOS (micro/fieldmul_bench.hip).
template <class C>
__device__ __forceinline__ Fp<C> mont_mul_dev(const Fp<C>& a, const Fp<C>& b) {
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
#endif

// Montgomery product a*b*R^{-1} mod P.  Device: FIPS (above).  Host: CIOS,
// no-carry variant.  Operands must be < P (the no-carry CIOS drops the top
// carry when an operand's high word is large; callers reduce unreduced
// 256-bit values with reduce_full / to_mont first).
template <class C>
QG_HD Fp<C> operator*(const Fp<C>& a, const Fp<C>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return mont_mul_dev<C>(a, b);
#endif
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.v[i];
    uint64_t A = (uint64_t)a.v[0] * bi + t[0];
    const uint32_t t0 = (uint32_t)A;
    const uint32_t m = t0 * C::INV;
    uint64_t Cc = (uint64_t)m * C::P[0] + t0;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      A = (uint64_t)a.v[j] * bi + t[j] + (A >> 32);
      Cc = (uint64_t)m * C::P[j] + (uint32_t)A + (Cc >> 32);
      t[j - 1] = (uint32_t)Cc;
    }
    t[7] = (uint32_t)(Cc >> 32) + (uint32_t)(A >> 32);
  }
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  reduce_once<C>(r.v);
  return r;
}

template <class C>
QG_HD Fp<C> fsqr(const Fp<C>& a) {
  return a * a;
}

// Montgomery -> canonical (multiply by 1)
template <class C>
QG_HD Fp<C> from_mont(const Fp<C>& a) {
  Fp<C> one = Fp<C>::zero();
  one.v[0] = 1;
  return a * one;
}

// t mod P for any t < 2^256 (both BN254 moduli exceed 2^256 / 5.3, so five
// conditional subtractions suffice)
template <class C>
QG_HD void reduce_full(uint32_t t[8]) {
#pragma unroll
  for (int k = 0; k < 5; k++) reduce_once<C>(t);
}

// canonical (< 2^256, may exceed P) -> Montgomery.  The operand is reduced
// first: the host CIOS product below loses its top carry for inputs >= P.
template <class C>
QG_HD Fp<C> to_mont(const Fp<C>& a) {
  Fp<C> r = a;
  reduce_full<C>(r.v);
  return r * Fp<C>::from_raw(C::R2);
}

template <class C>
QG_HD Fp<C> fpow_small(Fp<C> a, uint64_t e) {
  Fp<C> r = Fp<C>::one();
  while (e) {
    if (e & 1) r = r * a;
    a = fsqr(a);
    e >>= 1;
  }
  return r;
}

// a^(P-2): Fermat inversion (inverse of zero returns zero)
template <class C>
QG_HD Fp<C> finv_fermat(const Fp<C>& a) {
  // exponent P - 2, processed from the top bit down
  uint32_t e[8];
  uint32_t br = 0;
  e[0] = subb32(C::P[0], 2u, 0, &br);
#pragma unroll
  for (int i = 1; i < 8; i++) e[i] = subb32(C::P[i], 0u, br, &br);
  Fp<C> r = Fp<C>::one();
  for (int i = 7; i >= 0; i--) {
    for (int bit = 31; bit >= 0; bit--) {
      r = fsqr(r);
      if ((e[i] >> bit) & 1u) r = r * a;
    }
  }
  return r;
}

template <class C>
Fp<C> finv_host(const Fp<C>& a);  // bingcd.h (included at the end of this header)

// a^-1 (Montgomery in, Montgomery out; 0 -> 0).  Device: Fermat.  Host: the
// binary GCD of bingcd.h (~60x fewer operations than ~380 Montgomery products;
// the ML opening's host steps between two kernels run several per opening).
template <class C>
QG_HD Fp<C> finv(const Fp<C>& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return finv_fermat(a);
#else
  return finv_host(a);
#endif
}

// small integer -> Montgomery
template <class C>
QG_HD Fp<C> from_u64(uint64_t x) {
  Fp<C> t = Fp<C>::zero();
  t.v[0] = (uint32_t)x;
  t.v[1] = (uint32_t)(x >> 32);
  return to_mont(t);
}

// canonical compare: a > b (raw limbs)
QG_HD bool limbs_gt(const uint32_t* a, const uint32_t* b) {
  for (int i = 7; i >= 0; i--) {
    if (a[i] != b[i]) return a[i] > b[i];
  }
  return false;
}

}  // namespace qg

#include "bingcd.h"
