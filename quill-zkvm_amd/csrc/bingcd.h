// Modular inversion by binary GCD with 30-step approximated inner loops
// (T. Pornin, "Optimized Binary GCD for Modular Inversion", IACR ePrint
// 2020/972, Algorithm 2, with k = 31), host and device.
//
// Why: one field inversion per 2048-row block lets the Logup column run in ONE
// pass (logup.hip), and a Fermat inversion is ~380 dependent Montgomery
// products (~150 us on one lane).  Here: 17 outer iterations, each 30 cheap
// steps on 62-bit approximations of (a, b) that build a 2x2 matrix of 31-bit
// signed entries, then one full-width application of that matrix to (a, b)
// and, with an exact division by 2^30 folded in Montgomery-style, to (u, v).
//
// Invariants (mod P): a = y u, b = y v; a, b >= 0 (negated with their row of
// the matrix when the approximated steps overshoot).  After 2 len(P) - 1 = 507
// <= 17 * 30 steps a = 0 and b = gcd(y, P) = 1, so v = 1 / y.  y = 0 -> 0.
// Values are plain integers (no Montgomery factor), 8 x 32-bit limbs.
#pragma once
#include "field.h"

namespace qg {

namespace bgcd {

// (x f + y g) / 2^30 for x, y < 2^256 and |f| + |g| <= 2^30, exact division
// (the low 30 bits of x f + y g vanish); returns the sign, r = |result|
QG_HD bool lin_div30(const uint32_t* x, const uint32_t* y, int32_t f, int32_t g, uint32_t* r) {
  uint32_t t[9];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (int64_t)x[i] * f + (int64_t)y[i] * g;
    t[i] = (uint32_t)acc;
    acc >>= 32;  // arithmetic
  }
  t[8] = (uint32_t)acc;
  const bool neg = acc < 0;
#pragma unroll
  for (int i = 0; i < 8; i++) r[i] = (t[i] >> 30) | (t[i + 1] << 2);
  if (neg) {  // two's complement of the 8-limb value (magnitude < 2^254)
    uint32_t c = 1;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t s = ~r[i] + c;
      c = (c && s == 0) ? 1u : 0u;
      r[i] = s;
    }
  }
  return neg;
}

// (u f + v g) / 2^30 mod P for u, v < P, |f| + |g| <= 2^30: the division
// adds c P with c = -(u f + v g) / P mod 2^30 (pinv30 = P^-1 mod 2^30), the
// result lies in (-P, 2P) and is brought into [0, P)
template <class C>
QG_HD void lin_mod_div30(const uint32_t* u, const uint32_t* v, int32_t f, int32_t g, uint32_t pinv30,
                         uint32_t* r) {
  uint32_t t[9];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (int64_t)u[i] * f + (int64_t)v[i] * g;
    t[i] = (uint32_t)acc;
    acc >>= 32;
  }
  int64_t top = acc;  // signed top limb
  const uint32_t c = (0u - t[0] * pinv30) & 0x3fffffffu;
  uint64_t car = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint64_t s = (uint64_t)t[i] + (uint64_t)c * C::P[i] + car;
    t[i] = (uint32_t)s;
    car = s >> 32;
  }
  top += (int64_t)car;
  uint32_t q[8];
#pragma unroll
  for (int i = 0; i < 7; i++) q[i] = (t[i] >> 30) | (t[i + 1] << 2);
  q[7] = (t[7] >> 30) | ((uint32_t)top << 2);
  const bool neg = top < 0;
  // neg: value = q - 2^256 (two's complement), in (-P, 0): add P;
  // else value in [0, 2P): subtract P when >= P
  uint32_t s[8];
  if (neg) {
    uint64_t cc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t w = (uint64_t)q[i] + C::P[i] + cc;
      r[i] = (uint32_t)w;
      cc = w >> 32;
    }
  } else {
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = subb32(q[i], C::P[i], br, &br);
    // borrow out: q < P, keep q
#pragma unroll
    for (int i = 0; i < 8; i++) r[i] = br ? q[i] : s[i];
  }
}

QG_HD int bitlen8(const uint32_t* x) {
  for (int i = 7; i >= 0; i--)
    if (x[i]) return 32 * i + 32 - __builtin_clz(x[i]);
  return 0;
}

// bits [s, s + 32) of an 8-limb value (zero beyond the top)
QG_HD uint32_t bits32(const uint32_t* x, int s) {
  const int q = s >> 5, o = s & 31;
  const uint32_t lo = q < 8 ? x[q] : 0u, hi = q + 1 < 8 ? x[q + 1] : 0u;
  return o ? (lo >> o) | (hi << (32 - o)) : lo;
}

}  // namespace bgcd

// y^-1 mod P (plain integers, y < P; 0 -> 0)
template <class C>
QG_HD Fp<C> inv_bingcd(const Fp<C>& y) {
  using namespace bgcd;
  // P^-1 mod 2^30 by Newton iteration (P odd)
  uint32_t pinv = C::P[0];
#pragma unroll
  for (int i = 0; i < 4; i++) pinv *= 2u - C::P[0] * pinv;
  const uint32_t pinv30 = pinv & 0x3fffffffu;
  uint32_t a[8], b[8], u[8], v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    a[i] = y.v[i];
    b[i] = C::P[i];
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0u;
  }
  for (int it = 0; it < 17; it++) {  // 17 x 30 = 510 >= 2 * 254 - 1 steps
    int n = bitlen8(a);
    const int nb = bitlen8(b);
    n = n > nb ? n : nb;
    n = n > 62 ? n : 62;
    // 30 low bits + the 32 bits from n - 32: exact once n <= 62
    uint64_t ab = ((uint64_t)bits32(a, n - 32) << 30) | (a[0] & 0x3fffffffu);
    uint64_t bb = ((uint64_t)bits32(b, n - 32) << 30) | (b[0] & 0x3fffffffu);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    for (int j = 0; j < 30; j++) {
      if (ab & 1u) {
        if (ab < bb) {
          const uint64_t t = ab;
          ab = bb;
          bb = t;
          int32_t s = f0;
          f0 = f1;
          f1 = s;
          s = g0;
          g0 = g1;
          g1 = s;
        }
        ab -= bb;
        f0 -= f1;
        g0 -= g1;
      }
      ab >>= 1;
      f1 *= 2;
      g1 *= 2;
    }
    uint32_t na[8], nbv[8], nu[8], nv[8];
    if (lin_div30(a, b, f0, g0, na)) {
      f0 = -f0;
      g0 = -g0;
    }
    if (lin_div30(a, b, f1, g1, nbv)) {
      f1 = -f1;
      g1 = -g1;
    }
    lin_mod_div30<C>(u, v, f0, g0, pinv30, nu);
    lin_mod_div30<C>(u, v, f1, g1, pinv30, nv);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      a[i] = na[i];
      b[i] = nbv[i];
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  Fp<C> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = v[i];
  return r;
}

// Host finv (field.h): y = aR is inverted as a plain integer, z = (aR)^-1, and
// one Montgomery product by R^3 mod P gives a^-1 R.  One more product checks
// it (the iteration bound has little slack); Fermat if it ever did not converge.
template <class C>
inline Fp<C> finv_host(const Fp<C>& a) {
  if (a.is_zero()) return a;
  static const Fp<C> r3 = Fp<C>::from_raw(C::R2) * Fp<C>::from_raw(C::R2);  // R^3 mod P
  const Fp<C> r = inv_bingcd<C>(a) * r3;
  if (r * a == Fp<C>::one()) return r;
  return finv_fermat(a);
}

}  // namespace qg
