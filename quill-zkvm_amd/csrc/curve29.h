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

// madd-2008-s for a bucket accumulator kept lazily reduced between additions:
// X normalized < 16p, Y normalized < 8p, ZZ/ZZZ < 2p (x29_acc_finish brings
// it back to < 2p before it is stored).  Saves the X3/Y3 conditional
// subtractions of every addition.
QG_HD X29 x29_acc_madd(const X29& p, const A29& a) {
  if (x29_is_inf(p)) return x29_from_affine(a);
  const Q29 U2 = mul29(a.x, p.ZZ);
  const Q29 S2 = mul29(a.y, p.ZZZ);
  const Q29 P = normfull29(subk29(U2, p.X, F29P<FqP>::K17));  // (p, 19p)
  const Q29 R = normfull29(subk29(S2, p.Y, F29P<FqP>::K9));   // (p, 11p)
  if (is_zero_mod29_fast<FqP, 20>(P)) {
    if (is_zero_mod29_fast<FqP, 20>(R)) return x29_dbl_affine(a);
    return x29_inf();
  }
  const Q29 PP = sqr29(P);                 // < 3p
  const Q29 PPP = mul29(P, PP);            // < 2p
  const Q29 Q = mul29(p.X, PP);            // < 2p
  const Q29 X3 = normfull29(sub29(sub29(sub29(sqr29(R), PPP), Q), Q));  // < 16p
  const Q29 Y3 = normfull29(mulsub29(R, norm29(subk29(Q, X3, F29P<FqP>::K17)), p.Y, PPP));  // < 8p
  return {X3, Y3, mul29(p.ZZ, PP), mul29(p.ZZZ, PPP)};
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
