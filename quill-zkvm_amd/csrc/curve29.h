// BN254 G1 XYZZ arithmetic on the 29-bit-limb field (field29.h), R = 2^261.
// Same formulas as curve.h (madd-2008-s, add-2008-s, dbl-2008-s-1), with lazy
// additions: differences are carried un-normalized into the next multiply
// where the operand rules allow, and reduced below 2p (normalized) before
// they are stored, squared or compared.  Every output coordinate is
// normalized and < 2p.  Infinity: ZZ == 0 (all limbs), created explicitly.
#pragma once
#include "field29.h"

namespace qg {

using Q29 = F29<FqP>;

struct X29 {
  Q29 X, Y, ZZ, ZZZ;
};

struct A29 {
  Q29 x, y;
};

QG_HD X29 x29_inf() {
  return {Q29::zero(), Q29::from_l9(F29P<FqP>::ONE), Q29::zero(), Q29::zero()};
}

QG_HD bool x29_is_inf(const X29& p) { return is_zero29(p.ZZ); }

QG_HD X29 x29_from_affine(const A29& a) {
  const Q29 one = Q29::from_l9(F29P<FqP>::ONE);
  return {a.x, a.y, one, one};
}

// mdbl-2008-s-1: 2a for an affine point
QG_HD X29 x29_dbl_affine(const A29& a) {
  const Q29 U = normfull29(add29(a.y, a.y));  // < 4p
  const Q29 V = sqr29(U);
  const Q29 W = mul29(U, V);
  const Q29 S = mul29(a.x, V);
  const Q29 X2 = sqr29(a.x);
  const Q29 M = normfull29(add29(add29(X2, X2), X2));  // < 6p
  const Q29 X3 = red16p29(sub29(sub29(sqr29(M), S), S));
  const Q29 Y3 = red6p29(mulsub29(M, norm29(sub29(S, X3)), W, a.y));
  return {X3, Y3, V, W};
}

// dbl-2008-s-1
QG_HD X29 x29_dbl(const X29& p) {
  if (x29_is_inf(p)) return p;
  const Q29 U = normfull29(add29(p.Y, p.Y));
  const Q29 V = sqr29(U);
  const Q29 W = mul29(U, V);
  const Q29 S = mul29(p.X, V);
  const Q29 X2 = sqr29(p.X);
  const Q29 M = normfull29(add29(add29(X2, X2), X2));
  const Q29 X3 = red16p29(sub29(sub29(sqr29(M), S), S));
  const Q29 Y3 = red6p29(mulsub29(M, norm29(sub29(S, X3)), W, p.Y));
  return {X3, Y3, mul29(V, p.ZZ), mul29(W, p.ZZZ)};
}

// madd-2008-s: p + a (a affine, not infinity)
QG_HD X29 x29_add_affine(const X29& p, const A29& a) {
  if (x29_is_inf(p)) return x29_from_affine(a);
  const Q29 U2 = mul29(a.x, p.ZZ);
  const Q29 S2 = mul29(a.y, p.ZZZ);
  const Q29 P = normfull29(sub29(U2, p.X));  // value in (2p, 6p)
  const Q29 R = normfull29(sub29(S2, p.Y));
  if (is_zero_mod29_fast<FqP, 8>(P)) {
    if (is_zero_mod29_fast<FqP, 8>(R)) return x29_dbl_affine(a);
    return x29_inf();
  }
  const Q29 PP = sqr29(P);
  const Q29 PPP = mul29(P, PP);
  const Q29 Q = mul29(p.X, PP);
  const Q29 X3 = red16p29(sub29(sub29(sub29(sqr29(R), PPP), Q), Q));
  const Q29 Y3 = red6p29(mulsub29(R, norm29(sub29(Q, X3)), p.Y, PPP));
  return {X3, Y3, mul29(p.ZZ, PP), mul29(p.ZZZ, PPP)};
}

// ---- bucket accumulation (k_msm_accumulate) ---------------------------
// madd-2008-s (8M + 2S) on an accumulator kept lazily reduced between
// additions.  Invariants (values in units of p; 2^261 ~ 170 p):
//   X almost-normalized < 16p, Y normalized < 8p, ZZ / ZZZ normalized < 2p;
// the added point (x, y) is canonical (the table holds y and p - y, so a
// negative digit costs nothing).  Bounds (Montgomery output < a b / 170 + p):
//   U2 = x ZZ < 1.02, S2 = y ZZZ < 1.02,
//   P = U2 + 17p - X in (p, 18.1p) (normalized, zero-tested),
//   R = S2 + 9p - Y in (p, 10.1p) (almost-normalized),
//   PP < 3, PPP < 1.4, Q = X PP < 1.3, R^2 < 1.7,
//   X3 = R^2 + 12p - PPP - 2Q in (8p, 13.7p) < 16p (one parallel carry pass),
//   Y3 = R (Q + 17p - X3) - Y PPP + 4p < 10.1 * 18.3 / 170 + 5 < 6.1p < 8p
//   (mulsub output is normalized), ZZ3, ZZZ3 < 2p.
// Throughput multiplies (field29.h mul29t: one chain per column).  Returns
// false (accumulator untouched) when P == 0 mod p: the caller runs the
// exceptional cases (doubling / cancellation) off the main path.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ bool x29_acc_madd_tp(X29& p, const Q29& ax, const Q29& ay) {
#ifdef QG_MADD_SINGLE
  const Q29 U2 = mul29t(ax, p.ZZ);
  const Q29 S2 = mul29t(ay, p.ZZZ);
#else
  // independent products in interleaved pairs (field29.h mul29t2)
  Q29 U2, S2;
  mul29t2(ax, p.ZZ, ay, p.ZZZ, U2, S2);
#endif
  const Q29 P = normfull29(subk29(U2, p.X, F29P<FqP>::K17));
  if (is_zero_mod29_fast<FqP, 20>(P)) return false;
  const Q29 R = norm29(subk29(S2, p.Y, F29P<FqP>::K9));
#ifdef QG_MADD_SINGLE
  const Q29 PP = sqr29t(P);
  const Q29 RR = sqr29t(R);
  const Q29 PPP = mul29t(P, PP);
  const Q29 Q = mul29t(p.X, PP);
#else
  Q29 PP, RR, PPP, Q;
  sqr29t2(P, R, PP, RR);
  mul29t2(P, PP, p.X, PP, PPP, Q);
#endif
  const Q29 X3 = norm29(sub29(sub29(sub29(RR, PPP), Q), Q));
  const Q29 Y3 = mulsub29t(R, norm29(subk29(Q, X3, F29P<FqP>::K17)), p.Y, PPP);
#ifdef QG_MADD_SINGLE
  p.ZZ = mul29t(p.ZZ, PP);
  p.ZZZ = mul29t(p.ZZZ, PPP);
#else
  Q29 ZZ3, ZZZ3;
  mul29t2(p.ZZ, PP, p.ZZZ, PPP, ZZ3, ZZZ3);
  p.ZZ = ZZ3;
  p.ZZZ = ZZZ3;
#endif
  p.X = X3;
  p.Y = Y3;
  return true;
}
#elif defined(__HIP__)
__device__ bool x29_acc_madd_tp(X29& p, const Q29& ax, const Q29& ay);
#endif

// the exceptional cases of x29_acc_madd_tp (P == 0 mod p): the point equals
// the accumulator (R == 0: double it) or its negative (infinity -> *inf)
QG_HD void x29_acc_madd_exc(X29& p, const Q29& ax, const Q29& ay, bool* inf) {
  const Q29 S2 = mul29(ay, p.ZZZ);
  const Q29 R = normfull29(subk29(S2, p.Y, F29P<FqP>::K9));
  if (is_zero_mod29_fast<FqP, 20>(R)) {
    A29 a;
    a.x = ax;
    a.y = ay;  // canonical
    p = x29_dbl_affine(a);
  } else {
    *inf = true;
  }
}

// ---- MSM table rows (curve.h MsmPt) ----------------------------------------
// pack a canonical point (x, y < p, 29-bit limbs, R = 2^261) or infinity
QG_HD MsmPt msm_pt_pack(const Q29& x, const Q29& y, bool inf) {
  MsmPt r;
#pragma unroll
  for (int i = 0; i < 32; i++) r.w[i] = 0;
  if (inf) {
    r.w[27] = 1u;
    return r;
  }
  // p - y (y in (0, p): BN254 G1 has no point with y = 0)
  Q29 ny;
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t t = F29P<FqP>::P.v[i] - y.l[i] - br;
    br = t >> 31;
    ny.l[i] = i < 8 ? (t & M29) : t;
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r.w[i] = x.l[i];
    r.w[8 + i] = y.l[i];
    r.w[16 + i] = ny.l[i];
  }
  r.w[24] = x.l[8];
  r.w[25] = y.l[8];
  r.w[26] = ny.l[8];
  return r;
}

QG_HD bool msm_pt_unpack(const MsmPt& a, Q29& x, Q29& y) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.l[i] = a.w[i];
    y.l[i] = a.w[8 + i];
  }
  x.l[8] = a.w[24];
  y.l[8] = a.w[25];
  return (a.w[27] & 1u) != 0u;
}

#if defined(__HIP_DEVICE_COMPILE__)
// gather of one row for a signed digit: five aligned 16-B loads (80 of 128 B)
__device__ __forceinline__ bool msm_pt_load(const MsmPt* __restrict__ table, uint32_t idx,
                                            bool neg, Q29& x, Q29& y) {
  const uint4* row = reinterpret_cast<const uint4*>(table + idx);
  const uint4 x0 = row[0], x1 = row[1];
  const uint4 y0 = row[neg ? 4 : 2], y1 = row[neg ? 5 : 3];
  const uint4 top = row[6];
  x.l[0] = x0.x; x.l[1] = x0.y; x.l[2] = x0.z; x.l[3] = x0.w;
  x.l[4] = x1.x; x.l[5] = x1.y; x.l[6] = x1.z; x.l[7] = x1.w;
  y.l[0] = y0.x; y.l[1] = y0.y; y.l[2] = y0.z; y.l[3] = y0.w;
  y.l[4] = y1.x; y.l[5] = y1.y; y.l[6] = y1.z; y.l[7] = y1.w;
  x.l[8] = top.x;
  y.l[8] = neg ? top.z : top.y;
  return (top.w & 1u) != 0u;
}
#elif defined(__HIP__)
__device__ bool msm_pt_load(const MsmPt* __restrict__ table, uint32_t idx, bool neg, Q29& x,
                            Q29& y);
#endif

// XYZZ accumulator in its 29-bit limbs as stored by the bucket accumulation
// (144 B, no reduction or re-limbing at the store); readers finish it with
// x29_acc_finish
struct X29Raw {
  uint4 q[9];
};

QG_HD X29Raw x29_raw(const X29& p) {
  uint32_t w[36];
#pragma unroll
  for (int i = 0; i < 9; i++) {
    w[i] = p.X.l[i];
    w[9 + i] = p.Y.l[i];
    w[18 + i] = p.ZZ.l[i];
    w[27 + i] = p.ZZZ.l[i];
  }
  X29Raw r;
#pragma unroll
  for (int k = 0; k < 9; k++) r.q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  return r;
}

QG_HD X29 x29_unraw(const X29Raw& r) {
  uint32_t w[36];
#pragma unroll
  for (int k = 0; k < 9; k++) {
    w[4 * k] = r.q[k].x;
    w[4 * k + 1] = r.q[k].y;
    w[4 * k + 2] = r.q[k].z;
    w[4 * k + 3] = r.q[k].w;
  }
  X29 p;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    p.X.l[i] = w[i];
    p.Y.l[i] = w[9 + i];
    p.ZZ.l[i] = w[18 + i];
    p.ZZZ.l[i] = w[27 + i];
  }
  return p;
}

// lazily reduced accumulator -> every coordinate < 2p
QG_HD X29 x29_acc_finish(const X29& p) {
  if (x29_is_inf(p)) return p;
  return {red16p29(p.X), condsub29<FqP>(condsub29<FqP>(p.Y, F29P<FqP>::P4), F29P<FqP>::P2), p.ZZ,
          p.ZZZ};
}

// add-2008-s: p + q
QG_HD X29 x29_add(const X29& p, const X29& q) {
  if (x29_is_inf(p)) return q;
  if (x29_is_inf(q)) return p;
  const Q29 U1 = mul29(p.X, q.ZZ);
  const Q29 U2 = mul29(q.X, p.ZZ);
  const Q29 S1 = mul29(p.Y, q.ZZZ);
  const Q29 S2 = mul29(q.Y, p.ZZZ);
  const Q29 P = normfull29(sub29(U2, U1));
  const Q29 R = normfull29(sub29(S2, S1));
  if (is_zero_mod29_fast<FqP, 8>(P)) {
    if (is_zero_mod29_fast<FqP, 8>(R)) return x29_dbl(p);
    return x29_inf();
  }
  const Q29 PP = sqr29(P);
  const Q29 PPP = mul29(P, PP);
  const Q29 Q = mul29(U1, PP);
  const Q29 X3 = red16p29(sub29(sub29(sub29(sqr29(R), PPP), Q), Q));
  const Q29 Y3 = red6p29(mulsub29(R, norm29(sub29(Q, X3)), S1, PPP));
  return {X3, Y3, mul29(mul29(p.ZZ, q.ZZ), PP), mul29(mul29(p.ZZZ, q.ZZZ), PPP)};
}

QG_HD X29 x29_neg(const X29& p) {
  return {p.X, red6p29(sub29(Q29::zero(), p.Y)), p.ZZ, p.ZZZ};
}

// [k]p for a small scalar (double-and-add, top bit first)
QG_HD X29 x29_mul_small(const X29& p, uint32_t k) {
  X29 acc = x29_inf();
  for (int b = 31; b >= 0; b--) {
    acc = x29_dbl(acc);
    if ((k >> b) & 1u) acc = x29_add(acc, p);
  }
  return acc;
}

// HBM word layouts (8 x 32 per coordinate, values < 2p as plain integers)
QG_HD X29 x29_load(const G1Xyzz& w) { return {to29(w.X), to29(w.Y), to29(w.ZZ), to29(w.ZZZ)}; }
QG_HD G1Xyzz x29_store(const X29& p) { return {from29(p.X), from29(p.Y), from29(p.ZZ), from29(p.ZZZ)}; }

// affine word point in the R = 2^261 domain ((0,0) = infinity)
QG_HD A29 a29_load(const G1Affine& w) { return {to29(w.x), to29(w.y)}; }

// R = 2^261 -> R = 2^256 Montgomery words (canonical), for export
QG_HD Fq q29_export(const Q29& a) {
  return from29(canon29(mul29(a, Q29::from_l9(F29P<FqP>::TO256))));
}
// R = 2^256 Montgomery words -> R = 2^261 (canonical)
QG_HD Q29 q29_import(const Fq& a) {
  return canon29(mul29(to29(a), Q29::from_l9(F29P<FqP>::TO261)));
}

}  // namespace qg
