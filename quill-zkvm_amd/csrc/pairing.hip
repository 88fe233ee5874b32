// BN254 optimal ate pairing and the product-side verifiers (host C++).
//
// Replaces `E::pairing` of ark-bn254 0.5.0 (a crates.io dependency) at its one
// call site, KZG::verify (pcs/src/kzg.rs:98-108), and restates
// MLEvalProof::verify (pcs/src/mlpcs.rs:126-161) on top of it.  Verification
// is a handful of pairings per proof — latency, not throughput — so it runs on
// the host next to the transcript, with no device round trip.
//
// Tower: Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - xi), xi = 9 + u,
// Fq12 = Fq6[w]/(w^2 - v).  G2 is the D-type twist E'/Fq2: y^2 = x^3 + 3/xi,
// untwisted by (x, y) -> (x w^2, y w^3).  Miller loop over 6x + 2 (x = the BN
// parameter) in affine twisted coordinates: a line through T with twisted
// slope l evaluated at P = (xP, yP) is
//     yP + (-l xP) w + (l xT - yT) v w
// (vertical lines are dropped: they lie in Fq6 and die in the final
// exponentiation), followed by the lines with pi(Q) and -pi^2(Q).  Final
// exponentiation: f^(p^6 - 1) (conjugate / inverse), ^(p^2 + 1) (Frobenius),
// then the hard part (p^4 - p^2 + 1)/r by square-and-multiply.  The value is
// the reduced pairing f^((p^12 - 1)/r); ark-bn254's addition chain may return
// a fixed power of it, which no verification equation can observe.
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/quill_gpu.h"
#include "blake3.h"
#include "common.h"
#include "curve.h"

namespace qg {
namespace {

// ---------------------------------------------------------------- Fq2
struct Fq2 {
  Fq a, b;  // a + b u
  static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
  static Fq2 one() { return {Fq::one(), Fq::zero()}; }
  bool is_zero() const { return a.is_zero() && b.is_zero(); }
  bool operator==(const Fq2& o) const { return a == o.a && b == o.b; }
};
Fq2 operator+(const Fq2& x, const Fq2& y) { return {x.a + y.a, x.b + y.b}; }
Fq2 operator-(const Fq2& x, const Fq2& y) { return {x.a - y.a, x.b - y.b}; }
Fq2 neg(const Fq2& x) { return {fneg(x.a), fneg(x.b)}; }
Fq2 operator*(const Fq2& x, const Fq2& y) {
  // Karatsuba: (a0 a1 - b0 b1) + ((a0 + b0)(a1 + b1) - a0 a1 - b0 b1) u
  const Fq aa = x.a * y.a, bb = x.b * y.b;
  return {aa - bb, (x.a + x.b) * (y.a + y.b) - aa - bb};
}
Fq2 scale(const Fq2& x, const Fq& s) { return {x.a * s, x.b * s}; }
Fq2 conj(const Fq2& x) { return {x.a, fneg(x.b)}; }
Fq2 inv(const Fq2& x) {
  const Fq n = finv(x.a * x.a + x.b * x.b);
  return {x.a * n, fneg(x.b * n)};
}
Fq2 mul_xi(const Fq2& x) {  // (a + b u)(9 + u) = (9a - b) + (a + 9b) u
  const Fq nine = from_u64<FqP>(9);
  return {nine * x.a - x.b, x.a + nine * x.b};
}
Fq2 pow(Fq2 x, const uint32_t e[8]) {
  Fq2 r = Fq2::one();
  for (int i = 7; i >= 0; i--)
    for (int bit = 31; bit >= 0; bit--) {
      r = r * r;
      if ((e[i] >> bit) & 1u) r = r * x;
    }
  return r;
}

// ---------------------------------------------------------------- Fq6
struct Fq6 {
  Fq2 c0, c1, c2;  // c0 + c1 v + c2 v^2
  static Fq6 zero() { return {Fq2::zero(), Fq2::zero(), Fq2::zero()}; }
  static Fq6 one() { return {Fq2::one(), Fq2::zero(), Fq2::zero()}; }
  bool operator==(const Fq6& o) const { return c0 == o.c0 && c1 == o.c1 && c2 == o.c2; }
};
Fq6 operator+(const Fq6& x, const Fq6& y) { return {x.c0 + y.c0, x.c1 + y.c1, x.c2 + y.c2}; }
Fq6 operator-(const Fq6& x, const Fq6& y) { return {x.c0 - y.c0, x.c1 - y.c1, x.c2 - y.c2}; }
Fq6 neg(const Fq6& x) { return {neg(x.c0), neg(x.c1), neg(x.c2)}; }
Fq6 operator*(const Fq6& x, const Fq6& y) {
  // Karatsuba over v^3 = xi (6 Fq2 products)
  const Fq2 t0 = x.c0 * y.c0, t1 = x.c1 * y.c1, t2 = x.c2 * y.c2;
  const Fq2 r0 = t0 + mul_xi((x.c1 + x.c2) * (y.c1 + y.c2) - t1 - t2);
  const Fq2 r1 = (x.c0 + x.c1) * (y.c0 + y.c1) - t0 - t1 + mul_xi(t2);
  const Fq2 r2 = (x.c0 + x.c2) * (y.c0 + y.c2) - t0 - t2 + t1;
  return {r0, r1, r2};
}
Fq6 mul_v(const Fq6& x) { return {mul_xi(x.c2), x.c0, x.c1}; }
Fq6 inv(const Fq6& x) {
  const Fq2 A = x.c0 * x.c0 - mul_xi(x.c1 * x.c2);
  const Fq2 B = mul_xi(x.c2 * x.c2) - x.c0 * x.c1;
  const Fq2 C = x.c1 * x.c1 - x.c0 * x.c2;
  const Fq2 F = x.c0 * A + mul_xi(x.c2 * B) + mul_xi(x.c1 * C);
  const Fq2 Fi = inv(F);
  return {A * Fi, B * Fi, C * Fi};
}

// ---------------------------------------------------------------- Fq12
struct Fq12 {
  Fq6 c0, c1;  // c0 + c1 w
  static Fq12 one() { return {Fq6::one(), Fq6::zero()}; }
  bool operator==(const Fq12& o) const { return c0 == o.c0 && c1 == o.c1; }
};
Fq12 operator*(const Fq12& x, const Fq12& y) {
  const Fq6 t0 = x.c0 * y.c0, t1 = x.c1 * y.c1;
  return {t0 + mul_v(t1), (x.c0 + x.c1) * (y.c0 + y.c1) - t0 - t1};
}
Fq12 sqr(const Fq12& x) {
  // (c0 + c1 w)^2 = (c0^2 + v c1^2) + 2 c0 c1 w, complex-style
  const Fq6 t = x.c0 * x.c1;
  const Fq6 s = (x.c0 + x.c1) * (x.c0 + mul_v(x.c1)) - t - mul_v(t);
  return {s, t + t};
}
Fq12 conj(const Fq12& x) { return {x.c0, neg(x.c1)}; }
Fq12 inv(const Fq12& x) {
  const Fq6 d = inv(x.c0 * x.c0 - mul_v(x.c1 * x.c1));
  return {x.c0 * d, neg(x.c1 * d)};
}

// Frobenius constants gamma^k, gamma = xi^((p - 1)/6); the coefficient of w^k
// (k = i + 2j for c_i.c_j) maps to conj(.) gamma^k
struct Consts {
  Fq2 gamma[6];
  Fq2 b2;  // 3 / xi
  Consts() {
    uint32_t e[8], br = 0;
    e[0] = subb32(FqP::P[0], 1u, 0, &br);
    for (int i = 1; i < 8; i++) e[i] = subb32(FqP::P[i], 0u, br, &br);
    uint64_t rem = 0;
    for (int i = 7; i >= 0; i--) {  // (p - 1) / 6, exact
      const uint64_t cur = (rem << 32) | e[i];
      e[i] = (uint32_t)(cur / 6);
      rem = cur % 6;
    }
    gamma[0] = Fq2::one();
    gamma[1] = pow(Fq2{from_u64<FqP>(9), Fq::one()}, e);
    for (int k = 2; k < 6; k++) gamma[k] = gamma[k - 1] * gamma[1];
    b2 = Fq2{from_u64<FqP>(3), Fq::zero()} * inv(Fq2{from_u64<FqP>(9), Fq::one()});
  }
};
const Consts& K() {
  static const Consts k;
  return k;
}

Fq2* coef(Fq12& x, int k) {
  Fq6& c = (k & 1) ? x.c1 : x.c0;
  const int j = k >> 1;
  return j == 0 ? &c.c0 : (j == 1 ? &c.c1 : &c.c2);
}
Fq12 frob(const Fq12& x) {
  Fq12 r = x;
  for (int k = 0; k < 6; k++) *coef(r, k) = conj(*coef(r, k)) * K().gamma[k];
  return r;
}

// ---------------------------------------------------------------- G2 (affine, twisted)
struct G2A {
  Fq2 x, y;
  bool inf;
};
G2A g2_neg(const G2A& q) { return {q.x, neg(q.y), q.inf}; }
bool g2_on_curve(const G2A& q) { return q.inf || q.y * q.y == q.x * q.x * q.x + K().b2; }
G2A g2_add(const G2A& p, const G2A& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  Fq2 l;
  if (p.x == q.x) {
    if ((p.y + q.y).is_zero()) return {Fq2::zero(), Fq2::zero(), true};
    const Fq2 x2 = p.x * p.x;
    l = (x2 + x2 + x2) * inv(p.y + p.y);
  } else {
    l = (q.y - p.y) * inv(q.x - p.x);
  }
  const Fq2 x3 = l * l - p.x - q.x;
  return {x3, l * (p.x - x3) - p.y, false};
}
// k canonical (plain integer limbs)
G2A g2_mul(G2A q, const Fr& k) {
  G2A acc{Fq2::zero(), Fq2::zero(), true};
  for (int i = 7; i >= 0; i--)
    for (int bit = 31; bit >= 0; bit--) {
      acc = g2_add(acc, acc);
      if ((k.v[i] >> bit) & 1u) acc = g2_add(acc, q);
    }
  return acc;
}
G2A g2_frob(const G2A& q) {
  return {conj(q.x) * K().gamma[2], conj(q.y) * K().gamma[3], q.inf};
}

// ---------------------------------------------------------------- G1 helpers
G1Affine g1_mul(const G1Affine& p, const Fr& k) {  // k canonical
  G1Xyzz acc = G1Xyzz::infinity();
  for (int i = 7; i >= 0; i--)
    for (int bit = 31; bit >= 0; bit--) {
      acc = xyzz_dbl(acc);
      if ((k.v[i] >> bit) & 1u) acc = xyzz_add_affine(acc, p);
    }
  return xyzz_to_affine(acc);
}
G1Affine g1_add(const G1Affine& a, const G1Affine& b) {
  return xyzz_to_affine(xyzz_add_affine(G1Xyzz::from_affine(a), b));
}

// ---------------------------------------------------------------- Miller loop
// 6x + 2 = 29793968203157093288 (65 bits): bits from the top
std::vector<int> ate_bits() {
  // 6x + 2 = 2^64 + 11347224129447541672
  const uint64_t low = 11347224129447541672ull;
  std::vector<int> b;
  b.push_back(1);  // bit 64
  for (int i = 63; i >= 0; i--) b.push_back((int)((low >> i) & 1u));
  return b;
}

Fq12 line(const Fq2& l, const G2A& T, const G1Affine& P) {
  Fq12 r;
  r.c0 = {Fq2{P.y, Fq::zero()}, Fq2::zero(), Fq2::zero()};
  r.c1 = {neg(scale(l, P.x)), l * T.x - T.y, Fq2::zero()};
  return r;
}

// f with T <- T + Q (T != +-Q), the chord slope
void add_step(Fq12& f, G2A& T, const G2A& Q, const G1Affine& P) {
  QG_CHECK(!(T.x == Q.x), QG_ERR_ASSERT, "pairing: degenerate Miller addition");
  const Fq2 l = (Q.y - T.y) * inv(Q.x - T.x);
  f = f * line(l, T, P);
  const Fq2 x3 = l * l - T.x - Q.x;
  T = {x3, l * (T.x - x3) - T.y, false};
}

Fq12 miller_loop(const G1Affine& P, const G2A& Q) {
  if (P.is_inf() || Q.inf) return Fq12::one();
  static const std::vector<int> bits = ate_bits();
  Fq12 f = Fq12::one();
  G2A T = Q;
  for (size_t i = 1; i < bits.size(); i++) {
    const Fq2 x2 = T.x * T.x;
    const Fq2 l = (x2 + x2 + x2) * inv(T.y + T.y);
    f = sqr(f) * line(l, T, P);
    const Fq2 x3 = l * l - T.x - T.x;
    T = {x3, l * (T.x - x3) - T.y, false};
    if (bits[i]) add_step(f, T, Q, P);
  }
  const G2A Q1 = g2_frob(Q);
  const G2A Q2 = g2_neg(g2_frob(Q1));
  add_step(f, T, Q1, P);
  add_step(f, T, Q2, P);
  return f;
}

// (p^4 - p^2 + 1) / r, 761 bits, most significant 32-bit word first
const uint32_t HARD[24] = {
    0x01baaa71u, 0x0b0759adu, 0x331ec151u, 0x83177fafu, 0x6c0eb522u, 0xd5b12278u,
    0x4e529a58u, 0x61876f6bu, 0x3b1b1355u, 0xd189227du, 0x79581e16u, 0xf3fd90c6u,
    0x6b887d56u, 0xd5095f23u, 0xaaa441e3u, 0x954bcf8au, 0xdcc7b44cu, 0x87cdbacfu,
    0xf1154e7eu, 0x1da014fdu, 0x5abf5cc4u, 0xf49c36d4u, 0xe81bb482u, 0xccdf42b1u};

Fq12 final_exp(const Fq12& f) {
  Fq12 t = conj(f) * inv(f);   // ^(p^6 - 1)
  t = frob(frob(t)) * t;        // ^(p^2 + 1)
  Fq12 r = Fq12::one();
  for (int i = 0; i < (int)(sizeof(HARD) / 4); i++)
    for (int bit = 31; bit >= 0; bit--) {
      r = sqr(r);
      if ((HARD[i] >> bit) & 1u) r = r * t;
    }
  return r;
}

// ---------------------------------------------------------------- ABI conversions
Fq fq_in(const uint64_t v[4]) {
  Fq r;
  for (int i = 0; i < 4; i++) {
    r.v[2 * i] = (uint32_t)v[i];
    r.v[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
  return r;
}
void fq_out(const Fq& a, uint64_t v[4]) {
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
}
// Prime-order subgroup membership of a twist point: [r - 1] Q == -Q, i.e.
// [r] Q == O.  The twist's cofactor is not 1, and the Miller loop and the
// line non-degeneracy assume order r, so every G2 input is checked like ark's
// CanonicalDeserialize with Validate::Yes.  The check costs one 254-bit
// double-and-add (a few ms on the host); verifying keys repeat across calls,
// so the last few accepted points are remembered.
bool g2_in_subgroup(const G2A& q) {
  if (q.inf) return true;
  static std::mutex mu;
  static std::vector<std::vector<uint8_t>> seen;
  std::vector<uint8_t> key(2 * sizeof(Fq2));
  memcpy(key.data(), &q.x, sizeof(Fq2));
  memcpy(key.data() + sizeof(Fq2), &q.y, sizeof(Fq2));
  {
    std::lock_guard<std::mutex> g(mu);
    for (const auto& k : seen)
      if (k == key) return true;
  }
  const Fr rm1 = from_mont(Fr::zero() - Fr::one());  // r - 1, plain limbs
  const G2A t = g2_mul(q, rm1);
  const G2A nq = g2_neg(q);
  const bool ok = !t.inf && t.x == nq.x && t.y == nq.y;
  if (ok) {
    std::lock_guard<std::mutex> g(mu);
    if (seen.size() >= 16) seen.erase(seen.begin());
    seen.push_back(key);
  }
  return ok;
}

G2A g2_in(const uint64_t xy[16], uint8_t inf) {
  if (inf) return {Fq2::zero(), Fq2::zero(), true};
  G2A q{{fq_in(xy), fq_in(xy + 4)}, {fq_in(xy + 8), fq_in(xy + 12)}, false};
  QG_CHECK(g2_on_curve(q), QG_ERR_INVALID, "G2 point not on the twist curve");
  QG_CHECK(g2_in_subgroup(q), QG_ERR_INVALID, "G2 point not in the prime-order subgroup");
  return q;
}
void g2_out(const G2A& q, uint64_t xy[16], uint8_t* inf) {
  memset(xy, 0, 128);
  if (inf) *inf = q.inf ? 1 : 0;
  if (q.inf) return;
  fq_out(q.x.a, xy);
  fq_out(q.x.b, xy + 4);
  fq_out(q.y.a, xy + 8);
  fq_out(q.y.b, xy + 12);
}
G1Affine g1_in(const uint64_t xy[8], uint8_t inf) {
  const G1Affine a = g1_import(xy, inf);
  QG_CHECK(affine_on_curve(a), QG_ERR_INVALID, "G1 point not on the curve");
  return a;
}

struct Vk {
  G1Affine g1;
  G2A g2, g2_tau;
};
Vk vk_in(const qg_kzg_vk* vk) {
  return {g1_in(vk->g1_xy, 0), g2_in(vk->g2_xy, 0), g2_in(vk->g2_tau_xy, 0)};
}

// KZG::verify (kzg.rs:98-108): e(C - y g1, g2) == e(proof, g2_tau - x g2).
// Rearranged by bilinearity into one product with a shared final
// exponentiation and no G2 scalar multiplication:
//   e(C - y g1 + x proof, g2) * e(-proof, g2_tau) == 1
// (the same acceptance set: both sides equal e(proof, g2)^(tau - x) ...).
bool kzg_verify(const Vk& vk, const G1Affine& comm, const Fr& x, const Fr& y,
                const G1Affine& proof) {
  const G1Affine lhs = g1_add(g1_add(comm, affine_neg(g1_mul(vk.g1, from_mont(y)))),
                              g1_mul(proof, from_mont(x)));
  const Fq12 f = miller_loop(lhs, vk.g2) * miller_loop(affine_neg(proof), vk.g2_tau);
  return final_exp(f) == Fq12::one();
}

bool kzg_verify_abi(const Vk& vk, const G1Affine& comm, const qg_kzg_opening& op) {
  return kzg_verify(vk, comm, fr_import(op.x), fr_import(op.y),
                    g1_in(op.proof_xy, op.proof_inf));
}

// MLEvalProof::eval_pr (mlpcs.rs:52-63)
Fr eval_pr(const std::vector<Fr>& r, Fr x) {
  Fr acc = Fr::one();
  for (const Fr& ri : r) {
    acc = acc * (ri * x + (Fr::one() - ri));
    x = x * x;
  }
  return acc;
}

}  // namespace
}  // namespace qg

using namespace qg;

extern "C" {

int qg_g2_generator(uint64_t out_xy[16]) {
  if (!out_xy) return QG_ERR_INVALID;
  // the standard BN254 G2 generator (canonical coordinates)
  static const uint64_t c[16] = {
      0x46debd5cd992f6edull, 0x674322d4f75edaddull, 0x426a00665e5c4479ull, 0x1800deef121f1e76ull,
      0x97e485b7aef312c2ull, 0xf1aa493335a9e712ull, 0x7260bfb731fb5d25ull, 0x198e9393920d483aull,
      0x4ce6cc0166fa7daaull, 0xe3d1e7690c43d37bull, 0x4aab71808dcb408full, 0x12c85ea5db8c6debull,
      0x55acdadcd122975bull, 0xbc4b313370b38ef3ull, 0xec9e99ad690c3395ull, 0x090689d0585ff075ull};
  for (int k = 0; k < 4; k++) {
    Fq t;
    for (int i = 0; i < 4; i++) {
      t.v[2 * i] = (uint32_t)c[4 * k + i];
      t.v[2 * i + 1] = (uint32_t)(c[4 * k + i] >> 32);
    }
    fq_out(to_mont(t), out_xy + 4 * k);
  }
  return QG_OK;
}

int qg_g2_mul(const uint64_t xy[16], uint8_t inf, const uint64_t k[4], uint64_t out_xy[16],
              uint8_t* out_inf) {
  if (!xy || !k || !out_xy) return QG_ERR_INVALID;
  try {
    g2_out(g2_mul(g2_in(xy, inf), from_mont(fr_import(k))), out_xy, out_inf);
    return QG_OK;
  } catch (const Error& e) {
    return e.code;
  }
}

int qg_pairing(const uint64_t p_xy[8], uint8_t p_inf, const uint64_t q_xy[16], uint8_t q_inf,
               uint64_t out[48]) {
  if (!p_xy || !q_xy || !out) return QG_ERR_INVALID;
  try {
    Fq12 e = final_exp(miller_loop(g1_in(p_xy, p_inf), g2_in(q_xy, q_inf)));
    for (int k = 0; k < 6; k++) {
      // c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2 (each re, im)
      const Fq6& c = k < 3 ? e.c0 : e.c1;
      const Fq2& v = (k % 3 == 0) ? c.c0 : (k % 3 == 1 ? c.c1 : c.c2);
      fq_out(v.a, out + 8 * k);
      fq_out(v.b, out + 8 * k + 4);
    }
    return QG_OK;
  } catch (const Error& e) {
    return e.code;
  }
}

int qg_kzg_verify(const qg_kzg_vk* vk, const uint64_t comm_xy[8], uint8_t comm_inf,
                  const qg_kzg_opening* opening, int* ok) {
  if (!vk || !comm_xy || !opening || !ok) return QG_ERR_INVALID;
  try {
    *ok = kzg_verify_abi(vk_in(vk), g1_in(comm_xy, comm_inf), *opening) ? 1 : 0;
    return QG_OK;
  } catch (const Error& e) {
    return e.code;
  }
}

int qg_mle_verify(const qg_kzg_vk* vk, const uint64_t comm_xy[8], uint8_t comm_inf,
                  const uint64_t* point, size_t nvars, const qg_mle_proof* proof,
                  uint8_t state[32], int* ok) {
  if (!vk || !comm_xy || (!point && nvars) || !proof || !state || !ok) return QG_ERR_INVALID;
  try {
    const Vk v = vk_in(vk);
    const G1Affine comm = g1_in(comm_xy, comm_inf);
    const G1Affine s_comm = g1_in(proof->s_comm_xy, proof->s_comm_inf);
    // reconstruct the transcript (mlpcs.rs:133-140): point, evaluation, s_comm; draw r
    std::vector<Fr> r(nvars);
    std::vector<uint8_t> msg(8 + 32 * nvars);
    u64_to_bytes(nvars, msg.data());
    for (size_t i = 0; i < nvars; i++) {
      r[i] = fr_import(point + 4 * i);
      fr_to_bytes(r[i], msg.data() + 8 + 32 * i);
    }
    transcript_append(state, msg.data(), msg.size());
    uint8_t b32[32], b64[64];
    const Fr evaluation = fr_import(proof->evaluation);
    fr_to_bytes(evaluation, b32);
    transcript_append(state, b32, 32);
    g1_serialize(s_comm, b64);
    transcript_append(state, b64, 64);
    const Fr x = transcript_draw_fr(state);
    // r.inverse().unwrap() (mlpcs.rs:141)
    QG_CHECK(!x.is_zero(), QG_ERR_ASSERT, "challenge r = 0");
    const Fr x_inv = finv(x);
    // the four openings (mlpcs.rs:143-151), then the inner-product equation
    // (:153-160); like the reference, the openings' own x are not compared with r
    *ok = 0;
    if (!kzg_verify_abi(v, comm, proof->poly_opening) ||
        !kzg_verify_abi(v, comm, proof->poly_opening_inv) ||
        !kzg_verify_abi(v, s_comm, proof->s_opening) ||
        !kzg_verify_abi(v, s_comm, proof->s_opening_inv))
      return QG_OK;
    const Fr pr_r = eval_pr(r, x), pr_r_inv = eval_pr(r, x_inv);
    const Fr lhs = fr_import(proof->poly_opening.y) * pr_r_inv +
                   fr_import(proof->poly_opening_inv.y) * pr_r;
    const Fr rhs = x * fr_import(proof->s_opening.y) + x_inv * fr_import(proof->s_opening_inv.y) +
                   from_u64<FrP>(2) * evaluation;
    *ok = lhs == rhs ? 1 : 0;
    return QG_OK;
  } catch (const Error& e) {
    return e.code;
  }
}

}  // extern "C"
