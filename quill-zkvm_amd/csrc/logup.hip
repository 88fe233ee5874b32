// Logup log-derivative columns for gfx950 — replaces the per-row loops of
//   MultisetEqualityProof::prove  hyperplonk/src/piops/multiset_check.rs:43-95
//   SetInclusionProof::prove      hyperplonk/src/piops/set_inclusion.rs:93-131
// which evaluate h(x) through the expression tree for every row x, call
// (beta + h(x)).inverse().unwrap() 2^n times, and multiply by m(x) in subset
// mode.  Here: out[x] = m(x) / (beta + h(x)) in one HBM pass.
//
//  * Both expressions are compiled on the host into sums of monomials
//    (expr.h).  The coefficient of a monomial with f factors is pre-scaled by
//    2^(256 + 5f), so multiplying raw arkworks table entries (x 2^256) with
//    mul29 (x 2^-261) keeps both the denominator and the multiplier in
//    arkworks form; a coefficient that comes out as 2^261 (a bare table
//    entry) skips its multiply.
//  * Batch inversion (Montgomery's trick) at four levels, ONE field inversion
//    per column: phase 1 (k_logup_den) stores every row's beta + h(x) in the
//    output buffer and multiplies each block's rows together; phase 2
//    (k_logup_scan, one block) forms the exclusive prefix / suffix products of
//    the block products and their total, which the host inverts (binary GCD,
//    bingcd.h; on the device's scalar unit it took 50 us, more than the round
//    trip); phase 3 (k_logup) gives each block 1/(its product) = 1/total x
//    prefix x suffix, then within the block: each thread's running prefix of
//    its LG_K rows in registers (row values in LDS), wave shuffle scans of the
//    thread products, back-substitution.  mul29 drifts the power of two by -5
//    per product; every output is a product tree over the inverse and all other
//    rows, so one constant fixes all of them.
//  * k_logup_fused (QG_LOGUP_FUSED=1) is the one-pass alternative: one
//    binary-GCD inversion per 2048-row block, 128 instead of 192 B/row of HBM,
//    but slower - the column is VALU-bound and the block idles while wave 0
//    inverts (profiles/r03_logup_ab.txt).
//  * A zero denominator makes the block product zero: the kernel flags it and
//    the call returns QG_ERR_ASSERT (the reference panics in unwrap()).
//  * Per-block sums of the outputs feed SetInclusionProof's claimed sums
//    (set_inclusion.rs:162-166, 193-197) without a second pass.
#include <string.h>

#include <vector>

#include "bingcd.h"
#include "common.h"
#include "expr.h"
#include "field29.h"

using namespace qg;

namespace qg {

using R29 = F29<FrP>;

static constexpr int LG_BLOCK = 256;
static constexpr int LG_K = 8;                     // rows per thread
static constexpr int LG_ROWS = LG_BLOCK * LG_K;    // rows per block
static constexpr int LG_MAXM = 128;                // monomials per expression
static constexpr int LG_MAXF = 512;                // factor slots (both expressions)
static constexpr int LG_MAXT = 64;                 // distinct tables referenced

// device image of the two compiled expressions: [0] = beta + h, [1] = m
struct LgDev {
  uint32_t nm[2];
  uint32_t unit[2][LG_MAXM];  // coefficient is 2^261 (mul29 by it is the identity)
  uint32_t mlen[2][LG_MAXM];
  uint32_t fstart[2][LG_MAXM];
  L9 coef[2][LG_MAXM];
  uint32_t fac[LG_MAXF];
  const Fr* tab[LG_MAXT];
  L9 kinv;    // k_logup_fused: 2^778 mod r, mul29(P^-1, kinv) = block inverse (see there)
  L9 one256;  // 2^256 mod r: a padding row's denominator in the x 2^256 domain
};

// one expression at one row; < 2p, normalized
QG_DEV R29 lg_eval(const LgDev* __restrict__ g, int w, size_t row) {
  R29 acc = R29::zero();
  const uint32_t nm = g->nm[w];
  for (uint32_t m = 0; m < nm; m++) {
    const uint32_t len = g->mlen[w][m], fs = g->fstart[w][m];
    uint32_t j = 0;
    R29 t;
    if (g->unit[w][m]) {  // c 2^(base + 5f) = 2^261: the first factor as loaded (< p)
      t = to29(g->tab[g->fac[fs]][row]);
      j = 1;
    } else {
      t = R29::from_l9(g->coef[w][m]);
    }
    for (; j < len; j++) t = mul29(t, to29(g->tab[g->fac[fs + j]][row]));
    acc = red2p29(add29(acc, t));
  }
  return acc;
}

QG_DEV R29 shfl_up29(const R29& a, int d) {
  R29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = __shfl_up(a.l[i], d, 64);
  return r;
}
QG_DEV R29 shfl_down29(const R29& a, int d) {
  R29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = __shfl_down(a.l[i], d, 64);
  return r;
}

QG_DEV R29 lds_row(const uint32_t* vs, int k, int tid) {
  R29 v;
#pragma unroll
  for (int i = 0; i < 9; i++) v.l[i] = vs[(k * 9 + i) * LG_BLOCK + tid];
  return v;
}
QG_DEV void lds_put(uint32_t* vs, int k, int tid, const R29& v) {
#pragma unroll
  for (int i = 0; i < 9; i++) vs[(k * 9 + i) * LG_BLOCK + tid] = v.l[i];
}

// Phase 1: per row v = beta + h(row) (x 2^256), stored (< p) into the output
// buffer; the block's product of all its rows -> bprod[block].  A zero
// denominator makes the product zero (flagged).  128 threads x 16 rows per
// 2048-row block: 4096 waves at 2^22 rows, all resident in one round (256
// threads x 8 rows was 8192 waves for 6144 slots at 77 VGPRs: 1.33 rounds).
static constexpr int LG_DEN_BLOCK = 128;
static constexpr int LG_DEN_K = LG_ROWS / LG_DEN_BLOCK;
__global__ __launch_bounds__(LG_DEN_BLOCK) void k_logup_den(const LgDev* __restrict__ g, size_t n,
                                                            Fr* __restrict__ out,
                                                            Fr* __restrict__ bprod,
                                                            uint32_t* __restrict__ err) {
  __shared__ uint32_t wtot[LG_DEN_BLOCK / 64][9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const size_t base = (size_t)blockIdx.x * LG_ROWS + tid;
  const R29 one = R29::from_l9(F29P<FrP>::ONE);
  R29 T = one;
  bool zero = false;
  for (int k = 0; k < LG_DEN_K; k++) {
    const size_t row = base + (size_t)k * LG_DEN_BLOCK;
    if (row >= n) break;
    const R29 v = canon29(lg_eval(g, 0, row));
    zero |= is_zero29(v);
    out[row] = from29(v);
    T = mul29(T, v);
  }
  if (zero) atomicOr(err, 1u);
  for (int d = 32; d >= 1; d >>= 1) {
    const R29 o = shfl_down29(T, d);
    if (lane + d < 64) T = mul29(T, o);
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 9; i++) wtot[wv][i] = T.l[i];
  __syncthreads();
  if (tid == 0) {
    R29 p = one;
    for (int w = 0; w < LG_DEN_BLOCK / 64; w++) {
      R29 t;
#pragma unroll
      for (int i = 0; i < 9; i++) t.l[i] = wtot[w][i];
      p = mul29(p, t);
    }
    bprod[blockIdx.x] = from29(canon29(p));
  }
}

// Phase 2 (one block): exclusive prefix and suffix products of the nb block
// products, and their total (the single value the host inverts).  256 threads,
// one contiguous segment each (sequential products), wave shuffle scans of the
// segment products and the four wave totals: ~20 dependent products per
// thread at one wave per SIMD (a 1024-thread Hillis-Steele scan through LDS
// took 49 us at 2^22 rows).
static constexpr int LG_SCAN = 256;
__global__ __launch_bounds__(LG_SCAN) void k_logup_scan(const Fr* __restrict__ bprod, uint32_t nb,
                                                        Fr* __restrict__ pre, Fr* __restrict__ suf,
                                                        Fr* __restrict__ total) {
  __shared__ uint32_t wtot[LG_SCAN / 64][9];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t per = (nb + LG_SCAN - 1) / LG_SCAN;
  const uint32_t lo = tid * per < nb ? tid * per : nb, hi = lo + per < nb ? lo + per : nb;
  const R29 one = R29::from_l9(F29P<FrP>::ONE);
  R29 tp = one;  // product of this thread's segment
  for (uint32_t i = lo; i < hi; i++) tp = mul29(tp, to29(bprod[i]));
  R29 ip = tp, is = tp;  // inclusive in-wave prefix / suffix
  for (int d = 1; d < 64; d <<= 1) {
    const R29 a = shfl_up29(ip, d), b = shfl_down29(is, d);
    if (lane >= (uint32_t)d) ip = mul29(a, ip);
    if (lane + d < 64) is = mul29(is, b);
  }
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < 9; i++) wtot[wv][i] = ip.l[i];
  R29 ep = shfl_up29(ip, 1), es = shfl_down29(is, 1);
  if (lane == 0) ep = one;
  if (lane == 63) es = one;
  __syncthreads();
  R29 tot = one;
  for (uint32_t w = 0; w < LG_SCAN / 64; w++) {
    R29 t;
#pragma unroll
    for (int i = 0; i < 9; i++) t.l[i] = wtot[w][i];
    if (w < wv) ep = mul29(ep, t);
    if (w > wv) es = mul29(es, t);
    if (tid == 0) tot = mul29(tot, t);
  }
  if (tid == 0) *total = from29(canon29(tot));
  R29 rp = ep, rs = es;
  for (uint32_t k = 0; k < hi - lo; k++) {  // prefix up, suffix down, interleaved
    const uint32_t i = lo + k, j = hi - 1 - k;
    pre[i] = from29(canon29(rp));
    suf[j] = from29(canon29(rs));
    rp = mul29(rp, to29(bprod[i]));
    rs = mul29(rs, to29(bprod[j]));
  }
}

// Phase 3: 1/v for every row of the block from inv(total) x prefix x suffix of
// the block products (block inverse), then the thread-level Montgomery trick
// as in one pass: the rows' v values come back from the output buffer.
__global__ __launch_bounds__(LG_BLOCK) void k_logup(const LgDev* __restrict__ g, size_t n,
                                                    Fr* __restrict__ out,
                                                    const Fr* __restrict__ pre,
                                                    const Fr* __restrict__ suf,
                                                    const Fr* __restrict__ tinv,
                                                    Fr* __restrict__ bsum) {
  __shared__ uint32_t vs[LG_K * 9 * LG_BLOCK];  // row denominators, [k][limb][thread]
  __shared__ uint32_t wtot[LG_BLOCK / 64][9];
  __shared__ uint32_t wsum[LG_BLOCK / 64][9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const size_t base = (size_t)blockIdx.x * LG_ROWS + tid;
  const R29 one = R29::from_l9(F29P<FrP>::ONE);

  // 1. denominators back from HBM to LDS, then the running prefix of this thread's rows
  for (int k = 0; k < LG_K; k++) {
    const size_t row = base + (size_t)k * LG_BLOCK;
    const R29 v = row < n ? to29(out[row]) : one;
#pragma unroll
    for (int i = 0; i < 9; i++) vs[(k * 9 + i) * LG_BLOCK + tid] = v.l[i];
  }
  static_assert(LG_K == 8, "prefix chain is written out for 8 rows");
  R29 pre_r[LG_K];
  pre_r[0] = lds_row(vs, 0, tid);
  pre_r[1] = mul29(pre_r[0], lds_row(vs, 1, tid));
  pre_r[2] = mul29(pre_r[1], lds_row(vs, 2, tid));
  pre_r[3] = mul29(pre_r[2], lds_row(vs, 3, tid));
  pre_r[4] = mul29(pre_r[3], lds_row(vs, 4, tid));
  pre_r[5] = mul29(pre_r[4], lds_row(vs, 5, tid));
  pre_r[6] = mul29(pre_r[5], lds_row(vs, 6, tid));
  pre_r[7] = mul29(pre_r[6], lds_row(vs, 7, tid));
  const R29 T = pre_r[LG_K - 1];

  // 2. exclusive prefix / suffix products of T across the block (the two
  // scans' products as one interleaved pair, field29.h mul29tn)
  R29 ip = T, is = T;  // inclusive in-wave prefix / suffix
  for (int d = 1; d < 64; d <<= 1) {
    R29 x2[2] = {shfl_up29(ip, d), is}, y2[2] = {ip, shfl_down29(is, d)};
    mul29tn<FrP, 2>(x2, y2, x2);
    if (lane >= d) ip = x2[0];
    if (lane + d < 64) is = x2[1];
  }
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < 9; i++) wtot[wv][i] = ip.l[i];
  R29 ep = shfl_up29(ip, 1), es = shfl_down29(is, 1);
  if (lane == 0) ep = one;
  if (lane == 63) es = one;
  __syncthreads();
  for (int w = 0; w < LG_BLOCK / 64; w++) {  // wave products straight from LDS (uniform loop)
    R29 t;
#pragma unroll
    for (int i = 0; i < 9; i++) t.l[i] = wtot[w][i];
    if (w < wv) ep = mul29(ep, t);
    if (w > wv) es = mul29(es, t);
  }
  // 1 / (block product) = 1 / total x (other blocks' products)
  const R29 binv = mul29(mul29(to29(*tinv), to29(pre[blockIdx.x])), to29(suf[blockIdx.x]));
  R29 inv_run = mul29(mul29(binv, ep), es);  // 1 / T

  // 3. back-substitution: 1 / v_k overwrites v_k in LDS (own slots only);
  // the output product and the next running inverse as one interleaved pair
#define LG_BACK(k)                                                      \
  {                                                                     \
    R29 a2[2] = {inv_run, inv_run}, b2[2] = {pre_r[k - 1], lds_row(vs, k, tid)}; \
    mul29tn<FrP, 2>(a2, b2, a2);                                        \
    inv_run = a2[1];                                                    \
    lds_put(vs, k, tid, a2[0]);                                         \
  }
  LG_BACK(7) LG_BACK(6) LG_BACK(5) LG_BACK(4) LG_BACK(3) LG_BACK(2) LG_BACK(1)
#undef LG_BACK
  lds_put(vs, 0, tid, inv_run);

  // 4. multiplier (four rows' products interleaved), store, block sum
  R29 acc = R29::zero();
  for (int k0 = 0; k0 < LG_K; k0 += 4) {
    R29 xs[4], ms[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const size_t row = base + (size_t)(k0 + u) * LG_BLOCK;
      xs[u] = lds_row(vs, k0 + u, tid);
      ms[u] = row < n ? lg_eval(g, 1, row) : R29::zero();  // M x 2^256
    }
    mul29tn<FrP, 4>(xs, ms, xs);
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const size_t row = base + (size_t)(k0 + u) * LG_BLOCK;
      if (row >= n) break;
      const R29 y = canon29(xs[u]);
      out[row] = from29(y);
      acc = red2p29(add29(acc, y));
    }
  }
  // block sum (values < 2p; a wave tree then 4 wave partials)
  for (int d = 32; d >= 1; d >>= 1) {
    R29 o;
#pragma unroll
    for (int i = 0; i < 9; i++) o.l[i] = __shfl_xor(acc.l[i], d, 64);
    acc = red2p29(add29(acc, o));
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 9; i++) wsum[wv][i] = acc.l[i];
  __syncthreads();
  if (tid == 0) {
    R29 s = R29::zero();
#pragma unroll
    for (int w = 0; w < LG_BLOCK / 64; w++) {
      R29 t;
#pragma unroll
      for (int i = 0; i < 9; i++) t.l[i] = wsum[w][i];
      s = red2p29(add29(s, t));
    }
    bsum[blockIdx.x] = from29(canon29(s));
  }
}

// One pass (default): k_logup with the denominators evaluated from the tables
// instead of re-read, and 1 / (block product) from ONE binary-GCD inversion
// per 2048-row block (csrc/bingcd.h, wave 0 on the scalar unit) instead of a
// column-wide product inverted on the host: 96 B/row read + 32 B/row written,
// no scan kernel, no host round trip.
// Domains: the denominators stay in arkworks' x 2^256 form (the raw table
// entries add in without a conversion multiply; beta + t0 + a t1 costs one
// multiply).  Every mul29 takes 2^261 off, so a product of m such values
// carries 2^(261 - 5m); each 1 / v_k below is a product tree over binv and the
// block's other N - 1 rows, whatever its position, so with the block product P
// = (prod v) 2^(261 - 5N) inverted as a plain integer and binv = mul29(P^-1,
// 2^778) every 1 / v_k comes out as (1 / v_k) 2^261 - the multiplier's domain
// then gives the output in arkworks form.  (Padding rows are 2^256, i.e. 1.)
__global__ __launch_bounds__(LG_BLOCK) void k_logup_fused(const LgDev* __restrict__ g, size_t n,
                                                          Fr* __restrict__ out, Fr* __restrict__ bsum,
                                                          uint32_t* __restrict__ err) {
  __shared__ uint32_t vs[LG_K * 9 * LG_BLOCK];  // row denominators, [k][limb][thread]
  __shared__ uint32_t wtot[LG_BLOCK / 64][9];
  __shared__ uint32_t wsum[LG_BLOCK / 64][9];
  __shared__ uint32_t binv_sh[9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const size_t base = (size_t)blockIdx.x * LG_ROWS + tid;
  const R29 one = R29::from_l9(F29P<FrP>::ONE);

  // 1. denominators (x 2^261) into LDS, the running prefix of this thread's rows
  bool zero = false;
  for (int k = 0; k < LG_K; k++) {
    const size_t row = base + (size_t)k * LG_BLOCK;
    R29 v = R29::from_l9(g->one256);
    if (row < n) {
      v = canon29(lg_eval(g, 0, row));
      zero |= is_zero29(v);
    }
    lds_put(vs, k, tid, v);
  }
  if (zero) atomicOr(err, 1u);
  static_assert(LG_K == 8, "prefix chain is written out for 8 rows");
  R29 pre_r[LG_K];
  pre_r[0] = lds_row(vs, 0, tid);
  pre_r[1] = mul29(pre_r[0], lds_row(vs, 1, tid));
  pre_r[2] = mul29(pre_r[1], lds_row(vs, 2, tid));
  pre_r[3] = mul29(pre_r[2], lds_row(vs, 3, tid));
  pre_r[4] = mul29(pre_r[3], lds_row(vs, 4, tid));
  pre_r[5] = mul29(pre_r[4], lds_row(vs, 5, tid));
  pre_r[6] = mul29(pre_r[5], lds_row(vs, 6, tid));
  pre_r[7] = mul29(pre_r[6], lds_row(vs, 7, tid));
  const R29 T = pre_r[LG_K - 1];

  // 2. exclusive prefix / suffix products of T across the block
  R29 ip = T, is = T;
  for (int d = 1; d < 64; d <<= 1) {
    const R29 a = shfl_up29(ip, d), b = shfl_down29(is, d);
    if (lane >= d) ip = mul29(a, ip);
    if (lane + d < 64) is = mul29(is, b);
  }
  if (lane == 63)
#pragma unroll
    for (int i = 0; i < 9; i++) wtot[wv][i] = ip.l[i];
  R29 ep = shfl_up29(ip, 1), es = shfl_down29(is, 1);
  if (lane == 0) ep = one;
  if (lane == 63) es = one;
  __syncthreads();
  if (wv == 0) {  // block inverse: one binary-GCD inversion, wave-uniform (scalar unit)
    R29 P = one;
    for (int w = 0; w < LG_BLOCK / 64; w++) {
      R29 t;
#pragma unroll
      for (int i = 0; i < 9; i++) t.l[i] = wtot[w][i];
      P = mul29(P, t);
    }
    Fr pc = from29(canon29(P));
#pragma unroll
    for (int i = 0; i < 8; i++) pc.v[i] = __builtin_amdgcn_readfirstlane(pc.v[i]);
    const Fr ipl = inv_bingcd<FrP>(pc);  // 0 if some denominator was 0
    const R29 b = mul29(to29(ipl), R29::from_l9(g->kinv));
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 9; i++) binv_sh[i] = b.l[i];
  }
  for (int w = 0; w < LG_BLOCK / 64; w++) {  // wave products straight from LDS (uniform loop)
    R29 t;
#pragma unroll
    for (int i = 0; i < 9; i++) t.l[i] = wtot[w][i];
    if (w < wv) ep = mul29(ep, t);
    if (w > wv) es = mul29(es, t);
  }
  __syncthreads();
  R29 binv;
#pragma unroll
  for (int i = 0; i < 9; i++) binv.l[i] = binv_sh[i];
  R29 inv_run = mul29(mul29(binv, ep), es);  // 1 / T

  // 3. back-substitution: 1 / v_k overwrites v_k in LDS (own slots only)
#define LG_BACK(k)                                        \
  {                                                       \
    const R29 x = mul29(inv_run, pre_r[k - 1]);           \
    inv_run = mul29(inv_run, lds_row(vs, k, tid));        \
    lds_put(vs, k, tid, x);                               \
  }
  LG_BACK(7) LG_BACK(6) LG_BACK(5) LG_BACK(4) LG_BACK(3) LG_BACK(2) LG_BACK(1)
#undef LG_BACK
  lds_put(vs, 0, tid, inv_run);

  // 4. multiplier, store, block sum
  R29 acc = R29::zero();
  for (int k = 0; k < LG_K; k++) {
    const size_t row = base + (size_t)k * LG_BLOCK;
    if (row >= n) break;
    const R29 x = lds_row(vs, k, tid);
    const R29 m = lg_eval(g, 1, row);  // M x 2^256
    const R29 y = canon29(mul29(x, m));
    out[row] = from29(y);
    acc = red2p29(add29(acc, y));
  }
  for (int d = 32; d >= 1; d >>= 1) {
    R29 o;
#pragma unroll
    for (int i = 0; i < 9; i++) o.l[i] = __shfl_xor(acc.l[i], d, 64);
    acc = red2p29(add29(acc, o));
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 9; i++) wsum[wv][i] = acc.l[i];
  __syncthreads();
  if (tid == 0) {
    R29 s = R29::zero();
#pragma unroll
    for (int w = 0; w < LG_BLOCK / 64; w++) {
      R29 t;
#pragma unroll
      for (int i = 0; i < 9; i++) t.l[i] = wsum[w][i];
      s = red2p29(add29(s, t));
    }
    bsum[blockIdx.x] = from29(canon29(s));
  }
}

// sum of the per-block sums (one block)
__global__ __launch_bounds__(256) void k_logup_sum(const Fr* __restrict__ bsum, uint32_t nb,
                                                   Fr* __restrict__ res) {
  __shared__ uint32_t ws[4][9];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  R29 acc = R29::zero();
  for (uint32_t i = tid; i < nb; i += 256) acc = red2p29(add29(acc, to29(bsum[i])));
  for (int d = 32; d >= 1; d >>= 1) {
    R29 o;
#pragma unroll
    for (int i = 0; i < 9; i++) o.l[i] = __shfl_xor(acc.l[i], d, 64);
    acc = red2p29(add29(acc, o));
  }
  if (lane == 0)
#pragma unroll
    for (int i = 0; i < 9; i++) ws[wv][i] = acc.l[i];
  __syncthreads();
  if (tid == 0) {
    R29 s = R29::zero();
    for (int w = 0; w < 4; w++) {
      R29 t;
#pragma unroll
      for (int i = 0; i < 9; i++) t.l[i] = ws[w][i];
      s = red2p29(add29(s, t));
    }
    *res = from29(canon29(s));
  }
}

// qg_selftest_inverse's device path: one inversion per thread
template <class C>
__global__ void k_inv_selftest(const Fp<C>* __restrict__ in, Fp<C>* __restrict__ out, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = inv_bingcd<C>(in[i]);
}

template <class C>
static void inv_selftest(qg_ctx* ctx, bool dev, const uint64_t* in, uint64_t* out, size_t n) {
  std::vector<Fp<C>> h(n);
  for (size_t i = 0; i < n; i++)
    for (int l = 0; l < 4; l++) {
      h[i].v[2 * l] = (uint32_t)in[4 * i + l];
      h[i].v[2 * l + 1] = (uint32_t)(in[4 * i + l] >> 32);
    }
  for (size_t i = 0; i < n; i++) {
    Fp<C> t = h[i];
    reduce_full<C>(t.v);
    QG_CHECK(t == h[i], QG_ERR_INVALID, "inverse self-test input not canonical");
  }
  if (dev) {
    QG_CHECK(ctx, QG_ERR_INVALID, "device self-test needs a context");
    QG_HIP(hipSetDevice(ctx->device));
    Fp<C>* d = ctx->scratch_as<Fp<C>>("inv_selftest", 2 * n + 2);
    QG_HIP(hipMemcpyAsync(d, h.data(), n * sizeof(Fp<C>), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_inv_selftest<C>, dim3(div_up(n ? n : 1, 64)), dim3(64), 0, ctx->stream, d, d + n,
                       n);
    QG_LAUNCH_CHECK();
    QG_HIP(hipMemcpyAsync(h.data(), d + n, n * sizeof(Fp<C>), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
  } else {
    for (size_t i = 0; i < n; i++) h[i] = inv_bingcd<C>(h[i]);
  }
  for (size_t i = 0; i < n; i++)
    for (int l = 0; l < 4; l++)
      out[4 * i + l] = (uint64_t)h[i].v[2 * l] | ((uint64_t)h[i].v[2 * l + 1] << 32);
}

// first row whose expression value (slot 0, no beta) is nonzero; atomicMin
__global__ __launch_bounds__(256) void k_expr_first_nonzero(const LgDev* __restrict__ g, size_t n,
                                                            unsigned long long* first) {
  const size_t row = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (row >= n) return;
  const R29 v = canon29(lg_eval(g, 0, row));
  if (!is_zero29(v)) atomicMin(first, (unsigned long long)row);
}

// ---------------------------------------------------------------- host
static Fr lg_plain_mul(const Fr& x, const Fr& y) { return from_mont(to_mont(x) * to_mont(y)); }
static L9 lg_l9(const Fr& plain) {
  const R29 t = to29(plain);
  L9 r{};
  for (int i = 0; i < 9; i++) r.v[i] = t.l[i];
  return r;
}

// compile one expression into slot w of the image; `add_const` (Montgomery)
// is added to the constant monomial; `base` = 261 or 256 (output scale)
static void lg_compile(LgDev& d, int w, const SopProgram& sp, const Fr& add_const, bool with_const,
                       uint32_t base, std::vector<uint32_t>& tables_used, uint32_t& nfac) {
  std::vector<uint32_t> mlen = sp.mono_len;
  std::vector<Fr> coeff = sp.coeff;
  std::vector<std::vector<uint32_t>> facs;
  size_t off = 0;
  for (size_t m = 0; m < mlen.size(); m++) {
    std::vector<uint32_t> f;
    for (uint32_t j = 0; j < mlen[m]; j++) f.push_back(sp.used[sp.fac[off + j]]);
    off += mlen[m];
    facs.push_back(f);
  }
  if (with_const) {
    bool found = false;
    for (size_t m = 0; m < mlen.size(); m++)
      if (mlen[m] == 0) {
        coeff[m] = coeff[m] + add_const;
        found = true;
      }
    if (!found) {
      mlen.push_back(0);
      coeff.push_back(add_const);
      facs.push_back({});
    }
  }
  QG_CHECK(mlen.size() <= (size_t)LG_MAXM, QG_ERR_UNSUPPORTED, "logup expression has too many monomials");
  d.nm[w] = (uint32_t)mlen.size();
  for (size_t m = 0; m < mlen.size(); m++) {
    d.mlen[w][m] = mlen[m];
    d.fstart[w][m] = nfac;
    for (uint32_t t : facs[m]) {
      QG_CHECK(nfac < (uint32_t)LG_MAXF, QG_ERR_UNSUPPORTED, "logup expressions have too many factors");
      uint32_t slot = 0;
      while (slot < tables_used.size() && tables_used[slot] != t) slot++;
      if (slot == tables_used.size()) {
        QG_CHECK(slot < (uint32_t)LG_MAXT, QG_ERR_UNSUPPORTED, "logup expressions use too many tables");
        tables_used.push_back(t);
      }
      d.fac[nfac++] = slot;
    }
    const Fr cf = lg_plain_mul(from_mont(coeff[m]), pow2_mod_plain<FrP>(base + 5 * mlen[m]));
    d.coef[w][m] = lg_l9(cf);
    d.unit[w][m] = mlen[m] >= 1 && cf == pow2_mod_plain<FrP>(261) ? 1u : 0u;
  }
}

static size_t lg_local_size(const qg_ctx* ctx, uint32_t nvars) {
  uint32_t lw = 0;
  while ((1 << lw) < ctx->world) lw++;
  QG_CHECK((1 << lw) == ctx->world, QG_ERR_INVALID, "world size must be a power of two");
  QG_CHECK(nvars >= lw, QG_ERR_INVALID, "nvars must be at least log2(world)");
  QG_CHECK(nvars < 40, QG_ERR_INVALID, "nvars too large");
  return (size_t)1 << (nvars - lw);
}

// the 3-kernel path (default) or the one-pass kernel (QG_LOGUP_FUSED=1): one
// pass moves 128 instead of 192 B/row but idles the block during its
// inversion; the column is VALU-bound, so the 3 kernels are faster
// (profiles/r03_logup_ab.txt)
static bool logup_fused() {
  const char* ov = getenv("QG_LOGUP_FUSED");
  return ov && atoi(ov) != 0;
}

// the column sum (d_res) and the zero-denominator flag (d_err) of this rank,
// summed / or-ed over all ranks; QG_ERR_ASSERT when any rank had a zero
static Fr logup_total(qg_ctx* ctx, const Fr* d_res, const uint32_t* d_err) {
  struct {
    Fr res;
    uint32_t err;
  } h;
  QG_HIP(hipMemcpyAsync(&h.err, d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
  QG_HIP(hipMemcpyAsync(&h.res, d_res, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  if (h.err) h.res = Fr::zero();
  // every rank learns whether any rank hit a zero denominator, and the global sum
  struct {
    Fr s;
    uint32_t err, pad[7];
  } mine{h.res, h.err, {}};
  Fr total = Fr::zero();
  uint32_t any_err = 0;
  if (ctx->sharded) {
    uint8_t* d_g = ctx->scratch_as<uint8_t>("lg_gather", sizeof(mine) * (ctx->world + 1));
    QG_HIP(hipMemcpyAsync(d_g, &mine, sizeof(mine), hipMemcpyHostToDevice, ctx->stream));
    comm_allgather_bytes(ctx, d_g, d_g + sizeof(mine), sizeof(mine));
    std::vector<decltype(mine)> all(ctx->world);
    QG_HIP(hipMemcpyAsync(all.data(), d_g + sizeof(mine), sizeof(mine) * ctx->world,
                          hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    for (auto& a : all) {
      total = total + a.s;
      any_err |= a.err;
    }
  } else {
    total = h.res;
    any_err = h.err;
  }
  QG_CHECK(!any_err, QG_ERR_ASSERT, "logup denominator beta + h(x) is zero (reference: inverse().unwrap())");
  return total;
}

// out[x] = m(x) / (beta + h(x)) over this rank's rows; returns sum_x out[x]
// over all ranks (Fr, i.e. arkworks Montgomery words)
static Fr logup_run(qg_ctx* ctx, uint32_t nvars, uint32_t ntables, const std::vector<const Fr*>& tabs,
                    const qg_expr_op* hp, size_t hl, const uint64_t* hc, size_t hn,
                    const qg_expr_op* mp, size_t ml, const uint64_t* mc, size_t mn,
                    const uint64_t beta[4], Fr* d_out) {
  QG_CHECK(hp && hl, QG_ERR_INVALID, "missing h expression");
  const size_t n = lg_local_size(ctx, nvars);
  LgDev img;
  memset(&img, 0, sizeof(img));
  std::vector<uint32_t> used;
  uint32_t nfac = 0;
  try {
    const SopProgram sh = compile_program(hp, hl, hc, hn, ntables);
    // denominators in arkworks' x 2^256 form (raw t0 adds without a multiply;
    // the mul29 drift is one fixed power of two per output, see k_logup_fused)
    lg_compile(img, 0, sh, fr_import(beta), true, 256, used, nfac);
    if (mp && ml) {
      const SopProgram sm = compile_program(mp, ml, mc, mn, ntables);
      lg_compile(img, 1, sm, Fr::zero(), false, 256, used, nfac);
    } else {
      SopProgram one;
      lg_compile(img, 1, one, Fr::one(), true, 256, used, nfac);
    }
  } catch (const Error& e) {
    if (e.code != QG_ERR_UNSUPPORTED) throw;
    // outside the compiled envelope (more than 128 monomials, 512 factors or
    // 64 tables): materialise h (and m) with the generic interpreter, then run
    // the column over those tables with h = Input(0), m = Input(1)
    const bool has_m = mp && ml;
    Fr* ev = ctx->scratch_as<Fr>("lg_gen_tabs", n * (has_m ? 2 : 1));
    expr_table_device(ctx, n, ntables, tabs, hp, hl, hc, hn, ev);
    if (has_m) expr_table_device(ctx, n, ntables, tabs, mp, ml, mc, mn, ev + n);
    const qg_expr_op h0[1] = {{QG_OP_INPUT, 0}}, m1[1] = {{QG_OP_INPUT, 1}};
    std::vector<const Fr*> t2{ev};
    if (has_m) t2.push_back(ev + n);
    return logup_run(ctx, nvars, (uint32_t)t2.size(), t2, h0, 1, nullptr, 0, has_m ? m1 : nullptr,
                     has_m ? 1 : 0, nullptr, 0, beta, d_out);
  }
  for (size_t s = 0; s < used.size(); s++) img.tab[s] = tabs[used[s]];

  const uint32_t nb = div_up(n, LG_ROWS);
  uint8_t* io = ctx->scratch_as<uint8_t>("lg_io", sizeof(LgDev) + 64);
  LgDev* d_img = reinterpret_cast<LgDev*>(io);
  Fr* d_res = reinterpret_cast<Fr*>(io + sizeof(LgDev));
  uint32_t* d_err = reinterpret_cast<uint32_t*>(io + sizeof(LgDev) + 32);
  Fr* d_bsum = ctx->scratch_as<Fr>("lg_bsum", nb);
  // block products, their exclusive prefix / suffix products, total, 1/total
  Fr* d_bp = ctx->scratch_as<Fr>("lg_bprod", 3 * (size_t)nb + 2);
  Fr* d_pre = d_bp + nb;
  Fr* d_suf = d_pre + nb;
  Fr* d_tot = d_suf + nb;
  Fr* d_tinv = d_tot + 1;
  img.kinv = lg_l9(pow2_mod_plain<FrP>(778));
  img.one256 = lg_l9(pow2_mod_plain<FrP>(256));
  QG_HIP(hipMemcpyAsync(d_img, &img, sizeof(img), hipMemcpyHostToDevice, ctx->stream));
  QG_HIP(hipMemsetAsync(d_err, 0, 4, ctx->stream));
  if (logup_fused()) {
    {
      QgTimed tm(ctx, "logup_column");
      hipLaunchKernelGGL(k_logup_fused, dim3(nb), dim3(LG_BLOCK), 0, ctx->stream, d_img, n, d_out,
                         d_bsum, d_err);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_logup_sum, dim3(1), dim3(256), 0, ctx->stream, d_bsum, nb, d_res);
      QG_LAUNCH_CHECK();
    }
    return logup_total(ctx, d_res, d_err);
  }
  struct {
    Fr tot;
    uint32_t err;
  } ht;
  {
    // kernel time only: the timed region closes before the D2H copies and the sync
    QgTimed tm(ctx, "logup_column");
    hipLaunchKernelGGL(k_logup_den, dim3(nb), dim3(LG_DEN_BLOCK), 0, ctx->stream, d_img, n, d_out,
                       d_bp, d_err);
    QG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_logup_scan, dim3(1), dim3(LG_SCAN), 0, ctx->stream, d_bp, nb, d_pre,
                       d_suf, d_tot);
    QG_LAUNCH_CHECK();
  }
  QG_HIP(hipMemcpyAsync(&ht.tot, d_tot, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  QG_HIP(hipMemcpyAsync(&ht.err, d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  // one inversion for the whole column, of the product of every denominator:
  // with N rows in the x 2^256 domain, tot = P 2^(261 - 5N) (plain); each
  // 1 / v_k of k_logup is a product tree over tinv and the other N - 1 rows,
  // so tinv = tot^-1 2^517 gives every 1 / v_k as (1 / v_k) 2^261
  Fr tinv = Fr::zero();
  if (!ht.err) {
    const Fr tot_plain = ht.tot;  // nonzero: no denominator was zero
    Fr inv_plain = inv_bingcd<FrP>(tot_plain);
    // one multiply checks the binary GCD (its iteration bound has little
    // slack); Fermat inversion if it ever did not converge
    if (!(lg_plain_mul(tot_plain, inv_plain) == from_mont(Fr::one())))
      inv_plain = from_mont(finv(to_mont(tot_plain)));
    tinv = lg_plain_mul(inv_plain, pow2_mod_plain<FrP>(517));
  }
  if (!ht.err) {
    QG_HIP(hipMemcpyAsync(d_tinv, &tinv, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
    QgTimed tm(ctx, "logup_column");
    hipLaunchKernelGGL(k_logup, dim3(nb), dim3(LG_BLOCK), 0, ctx->stream, d_img, n, d_out, d_pre,
                       d_suf, d_tinv, d_bsum);
    QG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_logup_sum, dim3(1), dim3(256), 0, ctx->stream, d_bsum, nb, d_res);
    QG_LAUNCH_CHECK();
  }
  return logup_total(ctx, d_res, d_err);
}

}  // namespace qg

// ---------------------------------------------------------------- C-ABI
extern "C" {

int qg_logup_column(qg_ctx* ctx, uint32_t nvars, uint32_t ntables, const uint64_t* const* tables,
                    const qg_expr_op* h_prog, size_t h_len, const uint64_t* h_consts,
                    size_t h_nconsts, const qg_expr_op* m_prog, size_t m_len,
                    const uint64_t* m_consts, size_t m_nconsts, const uint64_t beta[4],
                    uint64_t* out, uint64_t out_sum[4]) {
  return qg_guard(ctx, [&] {
    QG_CHECK(ctx && beta && out, QG_ERR_INVALID, "null argument");
    QG_CHECK(ntables == 0 || tables, QG_ERR_INVALID, "null tables");
    const size_t n = lg_local_size(ctx, nvars);
    Fr* d = ctx->scratch_as<Fr>("lg_in", std::max<size_t>(1, n * (ntables + 1)));
    std::vector<const Fr*> tabs;
    for (uint32_t i = 0; i < ntables; i++) {
      QG_CHECK(tables[i] != nullptr, QG_ERR_INVALID, "null table");
      fr_upload(ctx, d + n * i, tables[i], n);
      tabs.push_back(d + n * i);
    }
    Fr* d_out = d + n * ntables;
    const Fr s = logup_run(ctx, nvars, ntables, tabs, h_prog, h_len, h_consts, h_nconsts, m_prog,
                           m_len, m_consts, m_nconsts, beta, d_out);
    fr_download(ctx, out, d_out, n);
    if (out_sum) fr_export(s, out_sum);
  });
}

int qg_logup_column_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables, const qg_buf* const* tables,
                        const qg_expr_op* h_prog, size_t h_len, const uint64_t* h_consts,
                        size_t h_nconsts, const qg_expr_op* m_prog, size_t m_len,
                        const uint64_t* m_consts, size_t m_nconsts, const uint64_t beta[4],
                        qg_buf* out, uint64_t out_sum[4]) {
  return qg_guard(ctx, [&] {
    QG_CHECK(ctx && beta && out, QG_ERR_INVALID, "null argument");
    QG_CHECK(ntables == 0 || tables, QG_ERR_INVALID, "null tables");
    const size_t n = lg_local_size(ctx, nvars);
    QG_CHECK(out->n >= n, QG_ERR_INVALID, "output buffer too short");
    std::vector<const Fr*> tabs;
    for (uint32_t i = 0; i < ntables; i++) {
      QG_CHECK(tables[i] && tables[i]->n >= n, QG_ERR_INVALID, "table buffer missing or too short");
      QG_CHECK(tables[i]->d != out->d, QG_ERR_INVALID, "output aliases an input table");
      tabs.push_back(tables[i]->d);
    }
    const Fr s = logup_run(ctx, nvars, ntables, tabs, h_prog, h_len, h_consts, h_nconsts, m_prog,
                           m_len, m_consts, m_nconsts, beta, out->d);
    if (out_sum) fr_export(s, out_sum);
  });
}

int qg_selftest_inverse(qg_ctx* ctx, int field, int on_device, const uint64_t* in, uint64_t* out,
                        size_t n) {
  if ((!in || !out) && n) return QG_ERR_INVALID;
  if (field != 0 && field != 1) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    if (field == 0) inv_selftest<FrP>(ctx, on_device != 0, in, out, n);
    else inv_selftest<FqP>(ctx, on_device != 0, in, out, n);
  });
}

// Circuit::check_constraints (transition_circuit.rs:153-172): first row x
// (this rank's block) with h(x) != 0, or -1.
int qg_expr_first_nonzero_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                              const qg_buf* const* tables, const qg_expr_op* prog, size_t len,
                              const uint64_t* consts, size_t nconsts, int64_t* first_row) {
  return qg_guard(ctx, [&] {
    QG_CHECK(ctx && prog && len && first_row, QG_ERR_INVALID, "null argument");
    QG_CHECK(ntables == 0 || tables, QG_ERR_INVALID, "null tables");
    const size_t n = lg_local_size(ctx, nvars);
    *first_row = -1;
    LgDev img;
    memset(&img, 0, sizeof(img));
    std::vector<uint32_t> used;
    uint32_t nfac = 0;
    bool generic = false;
    try {
      const SopProgram sp = compile_program(prog, len, consts, nconsts, ntables);
      if (sp.mono_len.empty()) return;  // identically zero
      // scale 256 + 5f: values come out in arkworks form (x 2^256); zero test only
      lg_compile(img, 0, sp, Fr::zero(), false, 256, used, nfac);
    } catch (const Error& e) {
      if (e.code != QG_ERR_UNSUPPORTED) throw;
      generic = true;
    }
    if (generic) {
      // h(x) materialised by the generic interpreter, then tested as Input(0)
      std::vector<const Fr*> tabs(ntables, nullptr);
      for (uint32_t i = 0; i < ntables; i++) {
        QG_CHECK(tables[i] && tables[i]->n >= n, QG_ERR_INVALID, "table buffer missing or too short");
        tabs[i] = tables[i]->d;
      }
      Fr* ev = ctx->scratch_as<Fr>("fnz_gen_tab", n);
      expr_table_device(ctx, n, ntables, tabs, prog, len, consts, nconsts, ev);
      memset(&img, 0, sizeof(img));
      used.clear();
      nfac = 0;
      const qg_expr_op h0[1] = {{QG_OP_INPUT, 0}};
      lg_compile(img, 0, compile_program(h0, 1, nullptr, 0, 1), Fr::zero(), false, 256, used, nfac);
      img.tab[0] = ev;
    } else {
      for (size_t s = 0; s < used.size(); s++) {
        QG_CHECK(tables[used[s]] && tables[used[s]]->n >= n, QG_ERR_INVALID,
                 "table buffer missing or too short");
        img.tab[s] = tables[used[s]]->d;
      }
    }
    uint8_t* io = ctx->scratch_as<uint8_t>("lg_io", sizeof(LgDev) + 64);
    LgDev* d_img = reinterpret_cast<LgDev*>(io);
    unsigned long long* d_first = reinterpret_cast<unsigned long long*>(io + sizeof(LgDev));
    const unsigned long long init = n;
    QG_HIP(hipMemcpyAsync(d_img, &img, sizeof(img), hipMemcpyHostToDevice, ctx->stream));
    QG_HIP(hipMemcpyAsync(d_first, &init, 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_expr_first_nonzero, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream,
                       d_img, n, d_first);
    QG_LAUNCH_CHECK();
    unsigned long long f = 0;
    QG_HIP(hipMemcpyAsync(&f, d_first, 8, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    *first_row = f >= n ? -1 : (int64_t)f;
  });
}

}  // extern "C"
