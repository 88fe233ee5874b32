// BN254 G1 (y^2 = x^3 + 3 over Fq) group law, host + device.
//
// Replaces the ark-ec 0.5.0 short-Weierstrass projective arithmetic used by
// `VariableBaseMSM::msm_unchecked` (call site pcs/src/kzg.rs:72).  Buckets use
// XYZZ coordinates (x = X/ZZ, y = Y/ZZZ, ZZ^3 = ZZZ^2): a mixed add costs 8M+2S
// and needs no field inversion.  Affine points in device memory encode the
// point at infinity as (0, 0), which is not on the curve (0 != 3).
#pragma once
#include "field.h"

namespace qg {

struct G1Affine {
  Fq x, y;
  QG_HD static G1Affine infinity() { return {Fq::zero(), Fq::zero()}; }
  QG_HD bool is_inf() const { return x.is_zero() && y.is_zero(); }
};

// One MSM window-table row (128 B = one HBM line): the affine point in the
// 9 x 29-bit-limb Montgomery domain of curve29.h (R = 2^261), canonical, with
// the negated point's y precomputed so a signed digit costs no arithmetic:
//   w[0..7] x limbs 0..7, w[8..15] y limbs 0..7, w[16..23] (p - y) limbs 0..7,
//   w[24] x limb 8, w[25] y limb 8, w[26] (p - y) limb 8,
//   w[27] flags (bit 0: the point at infinity; the limbs are then zero).
// A gather reads five 16-B aligned words: x, y or p - y, and the top limbs.
struct MsmPt {
  uint32_t w[32];
};

struct G1Xyzz {
  Fq X, Y, ZZ, ZZZ;
  QG_HD static G1Xyzz infinity() {
    return {Fq::zero(), Fq::one(), Fq::zero(), Fq::zero()};
  }
  QG_HD bool is_inf() const { return ZZ.is_zero(); }
  QG_HD static G1Xyzz from_affine(const G1Affine& a) {
    if (a.is_inf()) return infinity();
    return {a.x, a.y, Fq::one(), Fq::one()};
  }
};

// dbl-2008-s-1 (a = 0)
QG_HD G1Xyzz xyzz_dbl(const G1Xyzz& p) {
  if (p.is_inf()) return p;
  Fq U = fdbl(p.Y);
  Fq V = fsqr(U);
  Fq W = U * V;
  Fq S = p.X * V;
  Fq X2 = fsqr(p.X);
  Fq M = X2 + fdbl(X2);
  Fq X3 = fsqr(M) - fdbl(S);
  Fq Y3 = M * (S - X3) - W * p.Y;
  return {X3, Y3, V * p.ZZ, W * p.ZZZ};
}

// mdbl-2008-s-1: doubling of an affine point
QG_HD G1Xyzz xyzz_dbl_affine(const G1Affine& a) {
  Fq U = fdbl(a.y);
  Fq V = fsqr(U);
  Fq W = U * V;
  Fq S = a.x * V;
  Fq X2 = fsqr(a.x);
  Fq M = X2 + fdbl(X2);
  Fq X3 = fsqr(M) - fdbl(S);
  Fq Y3 = M * (S - X3) - W * a.y;
  return {X3, Y3, V, W};
}

// madd-2008-s: p + a (a affine, not infinity)
QG_HD G1Xyzz xyzz_add_affine(const G1Xyzz& p, const G1Affine& a) {
  if (a.is_inf()) return p;
  if (p.is_inf()) return G1Xyzz::from_affine(a);
  Fq U2 = a.x * p.ZZ;
  Fq S2 = a.y * p.ZZZ;
  Fq P = U2 - p.X;
  Fq R = S2 - p.Y;
  if (P.is_zero()) {
    if (R.is_zero()) return xyzz_dbl_affine(a);
    return G1Xyzz::infinity();
  }
  Fq PP = fsqr(P);
  Fq PPP = P * PP;
  Fq Q = p.X * PP;
  Fq X3 = fsqr(R) - PPP - fdbl(Q);
  Fq Y3 = R * (Q - X3) - p.Y * PPP;
  return {X3, Y3, p.ZZ * PP, p.ZZZ * PPP};
}

// add-2008-s: p + q
QG_HD G1Xyzz xyzz_add(const G1Xyzz& p, const G1Xyzz& q) {
  if (p.is_inf()) return q;
  if (q.is_inf()) return p;
  Fq U1 = p.X * q.ZZ;
  Fq U2 = q.X * p.ZZ;
  Fq S1 = p.Y * q.ZZZ;
  Fq S2 = q.Y * p.ZZZ;
  Fq P = U2 - U1;
  Fq R = S2 - S1;
  if (P.is_zero()) {
    if (R.is_zero()) return xyzz_dbl(p);
    return G1Xyzz::infinity();
  }
  Fq PP = fsqr(P);
  Fq PPP = P * PP;
  Fq Q = U1 * PP;
  Fq X3 = fsqr(R) - PPP - fdbl(Q);
  Fq Y3 = R * (Q - X3) - S1 * PPP;
  return {X3, Y3, p.ZZ * q.ZZ * PP, p.ZZZ * q.ZZZ * PPP};
}

QG_HD G1Xyzz xyzz_neg(const G1Xyzz& p) { return {p.X, fneg(p.Y), p.ZZ, p.ZZZ}; }

QG_HD G1Affine affine_neg(const G1Affine& a) {
  if (a.is_inf()) return a;
  return {a.x, fneg(a.y)};
}

// x = X/ZZ, y = Y/ZZZ (one inversion)
QG_HD G1Affine xyzz_to_affine(const G1Xyzz& p) {
  if (p.is_inf()) return G1Affine::infinity();
  Fq t = finv(p.ZZ * p.ZZZ);
  Fq zzinv = t * p.ZZZ;
  Fq zzzinv = t * p.ZZ;
  return {p.X * zzinv, p.Y * zzzinv};
}

// [k]p for a small scalar (double-and-add, top bit first)
QG_HD G1Xyzz xyzz_mul_small(const G1Xyzz& p, uint32_t k) {
  G1Xyzz acc = G1Xyzz::infinity();
  for (int b = 31; b >= 0; b--) {
    acc = xyzz_dbl(acc);
    if ((k >> b) & 1u) acc = xyzz_add(acc, p);
  }
  return acc;
}

QG_HD bool affine_on_curve(const G1Affine& a) {
  if (a.is_inf()) return true;
  Fq lhs = fsqr(a.y);
  Fq rhs = fsqr(a.x) * a.x + from_u64<FqP>(3);
  return lhs == rhs;
}

}  // namespace qg
