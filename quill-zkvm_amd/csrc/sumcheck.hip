// Sumcheck / zero-check prover for gfx950 — replaces
//   SumcheckProof::prove   hyperplonk/src/piops/sumcheck.rs:28-114
//   ZeroCheckProof::prove  hyperplonk/src/piops/zerocheck.rs:14-49
//   fast_eq_eval_hypercube hyperplonk/src/utils/eq_eval.rs:6-31
//   VirtualPolynomialStore::evaluate_poly / VirtualPolyExpr
//                          hyperplonk/src/utils/virtual_polynomial.rs:9-37,286-331
//
// Semantics kept from the reference: the round message is the coefficient-form
// polynomial sum_p h(g(2p) + X (g(2p+1) - g(2p))) with trailing zeros trimmed
// (ark-poly DensePolynomial), absorbed as u64 length + canonical coefficients;
// index bit 0 is bound first; challenges are LE(48 B) mod r.
//
// Device design (DESIGN.md "Sumcheck"):
//  * The expression tree is compiled on the host into a sum of monomials
//    (coefficient x product of inputs); the kernel evaluates it at t = 0..d
//    per pair with inputs advanced by additions (g(t+1) = g(t) + diff).
//  * Round j (j >= 1) fuses the fold by r_{j-1} with the round-j evaluation:
//    each thread reads 4 entries of every table, writes the 2 folded entries
//    and evaluates the pair they form — one HBM pass per round.
//  * Per-block partial sums -> a one-block "finish" kernel that sums them,
//    interpolates (inverse Vandermonde on t = 0..d), trims, serializes, runs the
//    BLAKE3 transcript on the device and writes r_j for the next fold.  No host
//    round trip inside the protocol.
//  * Once a table has <= 2^TAIL_LOG entries the remaining rounds run inside one
//    workgroup (fold + evaluate + transcript per round, synchronized by
//    barriers), removing 2 launches per round.
#include <string.h>

#include <algorithm>
#include <map>
#include <vector>

#include "blake3.h"
#include "common.h"

using namespace qg;

namespace qg {

static constexpr int SC_BLOCK = 256;
static constexpr int SC_MAX_BLOCKS = 1024;
static constexpr int TAIL_LOG = 8;   // single-workgroup tail once tables have <= 2^8 entries

// ---------------------------------------------------------------- programs
struct Mono {
  std::vector<uint32_t> fac;  // sorted input indices (with multiplicity)
  Fr coeff;
};

struct SopProgram {
  std::vector<uint32_t> used;    // original table index of each compact slot
  std::vector<uint32_t> mono_len;
  std::vector<uint32_t> fac;     // compact slot indices
  std::vector<Fr> coeff;
  std::vector<uint8_t> is_one;
  uint32_t degree = 0;           // max monomial degree
};

typedef std::map<std::vector<uint32_t>, Fr> PolyMap;

static PolyMap pm_add(const PolyMap& a, const PolyMap& b) {
  PolyMap r = a;
  for (auto& kv : b) {
    auto it = r.find(kv.first);
    if (it == r.end()) r[kv.first] = kv.second;
    else it->second = it->second + kv.second;
  }
  return r;
}

static PolyMap pm_mul(const PolyMap& a, const PolyMap& b, size_t cap) {
  PolyMap r;
  for (auto& x : a)
    for (auto& y : b) {
      std::vector<uint32_t> f = x.first;
      f.insert(f.end(), y.first.begin(), y.first.end());
      std::sort(f.begin(), f.end());
      Fr c = x.second * y.second;
      auto it = r.find(f);
      if (it == r.end()) r[f] = c;
      else it->second = it->second + c;
      QG_CHECK(r.size() <= cap, QG_ERR_UNSUPPORTED, "expression expands to too many monomials");
    }
  return r;
}

// syntactic degree (Mul adds, Add maxes, Input 1, Const 0) — sizes the outputs
static uint32_t expr_degree(const qg_expr_op* prog, size_t len) {
  std::vector<uint32_t> st;
  for (size_t i = 0; i < len; i++) {
    const uint32_t op = prog[i].op;
    if (op == QG_OP_INPUT) st.push_back(1);
    else if (op == QG_OP_CONST) st.push_back(0);
    else if (op == QG_OP_ADD || op == QG_OP_MUL) {
      QG_CHECK(st.size() >= 2, QG_ERR_INVALID, "malformed expression (stack underflow)");
      uint32_t b = st.back();
      st.pop_back();
      uint32_t a = st.back();
      st.pop_back();
      st.push_back(op == QG_OP_ADD ? std::max(a, b) : a + b);
    } else {
      throw Error(QG_ERR_INVALID, "unknown expression opcode");
    }
  }
  QG_CHECK(st.size() == 1, QG_ERR_INVALID, "malformed expression (stack size != 1)");
  return st[0];
}

static SopProgram compile_program(const qg_expr_op* prog, size_t len, const uint64_t* consts,
                                  size_t nconsts, uint32_t ntables) {
  std::vector<PolyMap> st;
  const size_t cap = 1024;
  for (size_t i = 0; i < len; i++) {
    const uint32_t op = prog[i].op, arg = prog[i].arg;
    if (op == QG_OP_INPUT) {
      QG_CHECK(arg < ntables, QG_ERR_INVALID, "expression input index out of range");
      PolyMap m;
      m[{arg}] = Fr::one();
      st.push_back(m);
    } else if (op == QG_OP_CONST) {
      QG_CHECK(arg < nconsts, QG_ERR_INVALID, "expression constant index out of range");
      PolyMap m;
      m[{}] = fr_import(consts + 4 * (size_t)arg);
      st.push_back(m);
    } else if (op == QG_OP_ADD || op == QG_OP_MUL) {
      QG_CHECK(st.size() >= 2, QG_ERR_INVALID, "malformed expression (stack underflow)");
      PolyMap b = st.back();
      st.pop_back();
      PolyMap a = st.back();
      st.pop_back();
      st.push_back(op == QG_OP_ADD ? pm_add(a, b) : pm_mul(a, b, cap));
    } else {
      throw Error(QG_ERR_INVALID, "unknown expression opcode");
    }
  }
  QG_CHECK(st.size() == 1, QG_ERR_INVALID, "malformed expression (stack size != 1)");
  SopProgram sp;
  std::map<uint32_t, uint32_t> slot;
  for (auto& kv : st[0]) {
    if (kv.second.is_zero()) continue;
    for (uint32_t t : kv.first)
      if (!slot.count(t)) slot[t] = 0;
  }
  for (auto& kv : slot) {
    kv.second = (uint32_t)sp.used.size();
    sp.used.push_back(kv.first);
  }
  for (auto& kv : st[0]) {
    if (kv.second.is_zero()) continue;
    sp.mono_len.push_back((uint32_t)kv.first.size());
    for (uint32_t t : kv.first) sp.fac.push_back(slot[t]);
    sp.coeff.push_back(kv.second);
    sp.is_one.push_back(kv.second == Fr::one() ? 1 : 0);
    sp.degree = std::max<uint32_t>(sp.degree, (uint32_t)kv.first.size());
  }
  return sp;
}

// device-side program image (read with uniform loads)
struct SopDev {
  uint32_t nmono;
  uint32_t nslots;
  uint32_t np;  // evaluation points = degree + 1
  uint32_t pad;
  uint32_t mono_len[256];
  uint8_t fac[1024];
  uint8_t is_one[256];
  Fr coeff[256];
  Fr vinv[16 * 16];  // inverse Vandermonde on nodes 0..np-1 (row = coefficient)
};

static void build_vinv(uint32_t np, Fr* out) {
  // coefficients of L_j(X) = prod_{m != j} (X - m) / (j - m), out[i*16 + j] = coeff_i(L_j)
  for (uint32_t i = 0; i < 16 * 16; i++) out[i] = Fr::zero();
  for (uint32_t j = 0; j < np; j++) {
    std::vector<Fr> poly(1, Fr::one());
    Fr den = Fr::one();
    for (uint32_t m = 0; m < np; m++) {
      if (m == j) continue;
      std::vector<Fr> np2(poly.size() + 1, Fr::zero());
      Fr negm = fneg(from_u64<FrP>(m));
      for (size_t k = 0; k < poly.size(); k++) {
        np2[k] = np2[k] + poly[k] * negm;
        np2[k + 1] = np2[k + 1] + poly[k];
      }
      poly = np2;
      Fr diff = (j >= m) ? from_u64<FrP>(j - m) : fneg(from_u64<FrP>(m - j));
      den = den * diff;
    }
    Fr dinv = finv(den);
    for (uint32_t i = 0; i < np; i++) out[i * 16 + j] = poly[i] * dinv;
  }
}

// ---------------------------------------------------------------- device math
// v[i] for a wave-uniform slot index i.  readfirstlane makes the index scalar
// so the switch lowers to scalar branches; a runtime-indexed register array
// would otherwise be demoted to scratch memory.
template <int K>
QG_DEV Fr sel(const Fr (&v)[K], uint32_t i) {
  i = __builtin_amdgcn_readfirstlane(i);
  switch (i) {
    case 0: return v[0];
    case 1: if constexpr (K > 1) return v[1]; else return v[0];
    case 2: if constexpr (K > 2) return v[2]; else return v[0];
    case 3: if constexpr (K > 3) return v[3]; else return v[0];
    case 4: if constexpr (K > 4) return v[4]; else return v[0];
    case 5: if constexpr (K > 5) return v[5]; else return v[0];
    case 6: if constexpr (K > 6) return v[6]; else return v[0];
    default: if constexpr (K > 7) return v[7]; else return v[0];
  }
}

// h(values) via the monomial program
template <int K>
QG_DEV Fr sop_eval(const SopDev* __restrict__ sp, const Fr (&val)[K]) {
  Fr acc = Fr::zero();
  uint32_t f = 0;
  const uint32_t nmono = sp->nmono;
  for (uint32_t m = 0; m < nmono; m++) {
    const uint32_t len = sp->mono_len[m];
    Fr prod;
    if (len == 0) {
      prod = sp->coeff[m];
    } else {
      prod = sel<K>(val, sp->fac[f]);
      for (uint32_t q = 1; q < len; q++) prod = prod * sel<K>(val, sp->fac[f + q]);
      if (!sp->is_one[m]) prod = prod * sp->coeff[m];
    }
    f += len;
    acc = acc + prod;
  }
  return acc;
}

struct TablePtrs {
  const Fr* src[8];
  Fr* dst[8];
};

// Load pair p (fold or not) of every slot -> low/diff
template <int K>
QG_DEV void load_pair(const TablePtrs& tp, uint32_t nslots, size_t p, bool fold, const Fr& r,
                      Fr (&lo)[K], Fr (&df)[K]) {
#pragma unroll
  for (int i = 0; i < K; i++) {
    if ((uint32_t)i < nslots) {
      Fr a, b;
      if (fold) {
        const Fr* s = tp.src[i] + 4 * p;
        Fr x0 = s[0], x1 = s[1], x2 = s[2], x3 = s[3];
        a = x0 + r * (x1 - x0);
        b = x2 + r * (x3 - x2);
        tp.dst[i][2 * p] = a;
        tp.dst[i][2 * p + 1] = b;
      } else {
        const Fr* s = tp.src[i] + 2 * p;
        a = s[0];
        b = s[1];
      }
      lo[i] = a;
      df[i] = b - a;
    } else {
      lo[i] = Fr::zero();
      df[i] = Fr::zero();
    }
  }
}

// Evaluation points t = T..NPMAX-1 by template recursion, so sums[] is only
// ever indexed by compile-time constants (a runtime-indexed accumulator array
// is demoted to scratch memory).
template <int T, int K, int NPMAX>
QG_DEV void eval_points(const SopDev* __restrict__ sp, uint32_t np, Fr (&lo)[K], const Fr (&df)[K],
                        Fr (&sums)[NPMAX]) {
  if constexpr (T < NPMAX) {
    if ((uint32_t)T < np) {
      if constexpr (T > 0) {
#pragma unroll
        for (int i = 0; i < K; i++) lo[i] = lo[i] + df[i];
      }
      sums[T] = sums[T] + sop_eval<K>(sp, lo);
      eval_points<T + 1, K, NPMAX>(sp, np, lo, df, sums);
    }
  }
}

template <int K, int NPMAX>
QG_DEV void eval_pair(const SopDev* __restrict__ sp, Fr (&lo)[K], const Fr (&df)[K],
                      Fr (&sums)[NPMAX]) {
  eval_points<0, K, NPMAX>(sp, sp->np, lo, df, sums);
}

QG_DEV Fr shfl_xor_fr(const Fr& a, int m) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __shfl_xor(a.v[i], m, 64);
  return r;
}

// block-wide sum of NPMAX field values (LDS scratch: (blockDim/64) * NPMAX Fr)
template <int NPMAX>
QG_DEV void block_sum(Fr (&s)[NPMAX], uint32_t np, Fr* lds) {
#pragma unroll
  for (int t = 0; t < NPMAX; t++) {
    if ((uint32_t)t < np) {
      for (int m = 32; m > 0; m >>= 1) s[t] = s[t] + shfl_xor_fr(s[t], m);
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++)
      if ((uint32_t)t < np) lds[wid * NPMAX + t] = s[t];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++) {
      if ((uint32_t)t < np) {
        Fr acc = lds[t];
        for (int w = 1; w < nw; w++) acc = acc + lds[w * NPMAX + t];
        s[t] = acc;
      }
    }
  }
  __syncthreads();
}

// round kernel: fused fold(r_{j-1}) + evaluate, per-block partial sums
template <int K, int NPMAX>
__global__ void __launch_bounds__(SC_BLOCK)
    k_sc_round(TablePtrs tp, const SopDev* __restrict__ sp, size_t npairs, int fold,
               const Fr* __restrict__ chal, Fr* __restrict__ partial) {
  __shared__ Fr lds[(SC_BLOCK / 64) * NPMAX];
  const uint32_t nslots = sp->nslots, np = sp->np;
  Fr r = fold ? *chal : Fr::zero();
  Fr sums[NPMAX];
#pragma unroll
  for (int t = 0; t < NPMAX; t++) sums[t] = Fr::zero();
  for (size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x; p < npairs;
       p += (size_t)gridDim.x * blockDim.x) {
    Fr lo[K], df[K];
    load_pair<K>(tp, nslots, p, fold != 0, r, lo, df);
    eval_pair<K, NPMAX>(sp, lo, df, sums);
  }
  block_sum<NPMAX>(sums, np, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++)
      if ((uint32_t)t < np) partial[(size_t)blockIdx.x * NPMAX + t] = sums[t];
  }
}

// Round bookkeeping shared by the finish and tail kernels (whole block):
// interpolate evals -> coefficients (lane t computes coefficient t), trim,
// serialize into an LDS word buffer, then one lane runs the word-oriented
// BLAKE3 transcript (absorb message, draw r_j).
struct RoundOut {
  uint32_t* state;       // 8-word (32 B) transcript state (device)
  Fr* chal;              // nvars challenges
  Fr* coeffs;            // nvars x width
  uint32_t* lens;        // nvars
  uint32_t width;        // row width (>= np)
};

struct FinishSmem {
  Fr ev[16];
  uint32_t msg[8 + 2 + 16 * 8];  // state || u64 len || coefficients (canonical LE)
  uint32_t chin[12];             // new state || "challenge"
  uint32_t ab[20];               // new state || 48 challenge bytes
  uint32_t len;
};

// LDS word source for b3_chunk_words (dynamic indices stay in LDS, not scratch)
struct LdsSrc {
  const uint32_t* p;
  QG_DEV uint32_t operator()(uint32_t i) const { return p[i]; }
};

QG_DEV void finish_round_block(const SopDev* __restrict__ sp, FinishSmem& sm, const RoundOut& ro,
                               uint32_t j) {
  const uint32_t np = sp->np, t = threadIdx.x;
  if (t == 0) sm.len = 0;
  if (t < 8) sm.msg[t] = ro.state[t];
  __syncthreads();
  if (t < ro.width) {
    Fr co = Fr::zero();
    if (t < np) {
      for (uint32_t u = 0; u < np; u++) co = co + sp->vinv[t * 16 + u] * sm.ev[u];
      Fr c = from_mont(co);
#pragma unroll
      for (int i = 0; i < 8; i++) sm.msg[10 + 8 * t + i] = c.v[i];
      if (!co.is_zero()) atomicMax(&sm.len, t + 1);
    }
    ro.coeffs[(size_t)j * ro.width + t] = co;  // trailing entries are zero by construction
  }
  __syncthreads();
  if (t == 0) {
    const uint32_t len = sm.len;
    sm.msg[8] = len;
    sm.msg[9] = 0;
    // state' = B3(state || msg)
    b3_chunk_words(LdsSrc{sm.msg}, 40 + 32 * len, sm.chin, 8);
    // challenge = B3-XOF(state' || "challenge")[0..48]
    sm.chin[8] = 0x6c616863u;  // "chal"
    sm.chin[9] = 0x676e656cu;  // "leng"
    sm.chin[10] = 0x00000065u; // "e"
#pragma unroll
    for (int i = 0; i < 8; i++) sm.ab[i] = sm.chin[i];
    b3_chunk_words(LdsSrc{sm.chin}, 41, sm.ab + 8, 12);
    // state'' = B3(state' || challenge)
    b3_chunk_words(LdsSrc{sm.ab}, 80, sm.chin, 8);
#pragma unroll
    for (int i = 0; i < 8; i++) ro.state[i] = sm.chin[i];
    Fr lo, hi;
#pragma unroll
    for (int i = 0; i < 8; i++) lo.v[i] = sm.ab[8 + i];
#pragma unroll
    for (int i = 0; i < 4; i++) hi.v[i] = sm.ab[16 + i];
#pragma unroll
    for (int i = 4; i < 8; i++) hi.v[i] = 0;
    ro.chal[j] = lo * Fr::from_raw(FrP::R2) + hi * Fr::from_raw(FrP::R3);
    ro.lens[j] = len;
  }
  __syncthreads();
}

template <int NPMAX>
QG_DEV void stash_evals(const Fr (&s)[NPMAX], uint32_t np, FinishSmem& sm) {
  if (threadIdx.x == 0) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++)
      if ((uint32_t)t < np) sm.ev[t] = s[t];
  }
}

template <int NPMAX>
__global__ void __launch_bounds__(SC_BLOCK)
    k_sc_finish(const SopDev* __restrict__ sp, const Fr* __restrict__ partial, uint32_t nblocks,
                RoundOut ro, uint32_t j) {
  __shared__ Fr lds[(SC_BLOCK / 64) * NPMAX];
  __shared__ FinishSmem sm;
  const uint32_t np = sp->np;
  Fr s[NPMAX];
#pragma unroll
  for (int t = 0; t < NPMAX; t++) s[t] = Fr::zero();
  for (uint32_t b = threadIdx.x; b < nblocks; b += blockDim.x) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++)
      if ((uint32_t)t < np) s[t] = s[t] + partial[(size_t)b * NPMAX + t];
  }
  block_sum<NPMAX>(s, np, lds);
  stash_evals<NPMAX>(s, np, sm);
  finish_round_block(sp, sm, ro, j);
}

// Remaining rounds j0..nvars-1 in one workgroup, then the final fold + claim.
// bufs: ping-pong scratch per slot (a: size >= 2^(n-j0-1), b: >= 2^(n-j0-2)).
template <int K, int NPMAX>
__global__ void __launch_bounds__(SC_BLOCK)
    k_sc_tail(TablePtrs tp0, TablePtrs bufA, TablePtrs bufB, const SopDev* __restrict__ sp,
              uint32_t nvars, uint32_t j0, int fold0, RoundOut ro, Fr* __restrict__ final_vals,
              Fr* __restrict__ evaluation) {
  __shared__ Fr lds[(SC_BLOCK / 64) * NPMAX];
  __shared__ FinishSmem sm;
  const uint32_t nslots = sp->nslots, np = sp->np;
  TablePtrs cur = tp0;
  int fold = fold0;
  for (uint32_t j = j0; j < nvars; j++) {
    const size_t npairs = (size_t)1 << (nvars - 1 - j);
    Fr r = fold ? ro.chal[j - 1] : Fr::zero();
    Fr sums[NPMAX];
#pragma unroll
    for (int t = 0; t < NPMAX; t++) sums[t] = Fr::zero();
    for (size_t p = threadIdx.x; p < npairs; p += blockDim.x) {
      Fr lo[K], df[K];
      load_pair<K>(cur, nslots, p, fold != 0, r, lo, df);
      eval_pair<K, NPMAX>(sp, lo, df, sums);
    }
    block_sum<NPMAX>(sums, np, lds);
    stash_evals<NPMAX>(sums, np, sm);
    finish_round_block(sp, sm, ro, j);
    // the folded tables written this round become the next source
    TablePtrs nxt;
    const TablePtrs& w = ((j - j0) & 1) ? bufB : bufA;
    for (int i = 0; i < 8; i++) {
      nxt.src[i] = fold ? cur.dst[i] : cur.src[i];
      nxt.dst[i] = w.dst[i];
    }
    // when round j did not fold (j == 0), its source stays the source
    cur = nxt;
    fold = 1;
  }
  // final fold with r_{n-1}: cur.src has 2 entries per slot
  if (threadIdx.x == 0) {
    Fr r = ro.chal[nvars - 1];
    Fr val[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
      if ((uint32_t)i < nslots) {
        Fr a = cur.src[i][0], b = cur.src[i][1];
        val[i] = a + r * (b - a);
        final_vals[i] = val[i];
      } else {
        val[i] = Fr::zero();
      }
    }
    *evaluation = sop_eval<K>(sp, val);
  }
}

// eq(bin(i), z) for i < 2^nbits over z[off .. off+nbits)   (eq_eval.rs:6-31)
__global__ void k_eq_small(const Fr* __restrict__ z, uint32_t off, uint32_t nbits,
                           Fr* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ((size_t)1 << nbits)) return;
  Fr acc = Fr::one();
  for (uint32_t j = 0; j < nbits; j++) {
    Fr zj = z[off + j];
    acc = acc * (((i >> j) & 1) ? zj : (Fr::one() - zj));
  }
  out[i] = acc;
}

__global__ void k_eq_combine(const Fr* __restrict__ low, const Fr* __restrict__ high,
                             uint32_t lbits, size_t n, Fr* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  out[i] = low[i & (((size_t)1 << lbits) - 1)] * high[i >> lbits];
}

// multi-GPU: sum this rank's block partials -> loc[0..np)
template <int NPMAX>
__global__ void __launch_bounds__(SC_BLOCK)
    k_sc_local_sum(const SopDev* __restrict__ sp, const Fr* __restrict__ partial, uint32_t nblocks,
                   Fr* __restrict__ loc) {
  __shared__ Fr lds[(SC_BLOCK / 64) * NPMAX];
  const uint32_t np = sp->np;
  Fr s[NPMAX];
#pragma unroll
  for (int t = 0; t < NPMAX; t++) s[t] = Fr::zero();
  for (uint32_t b = threadIdx.x; b < nblocks; b += blockDim.x) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++)
      if ((uint32_t)t < np) s[t] = s[t] + partial[(size_t)b * NPMAX + t];
  }
  block_sum<NPMAX>(s, np, lds);
  if (threadIdx.x == 0) {
#pragma unroll
    for (int t = 0; t < NPMAX; t++) loc[t] = (uint32_t)t < np ? s[t] : Fr::zero();
  }
}

// multi-GPU: fold each slot's last local pair with r (size 2 -> 1)
__global__ void k_sc_fold_last(TablePtrs cur, uint32_t nslots, const Fr* __restrict__ chal,
                               Fr* __restrict__ out) {
  const uint32_t i = threadIdx.x;
  if (i >= nslots) return;
  const Fr r = *chal;
  const Fr a = cur.src[i][0], b = cur.src[i][1];
  out[i] = a + r * (b - a);
}

// gathered [rank][slot] -> per-slot tables [slot][rank]
__global__ void k_sc_transpose(const Fr* __restrict__ in, uint32_t world, uint32_t nslots,
                               Fr* __restrict__ out) {
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= world * nslots) return;
  const uint32_t rk = idx / nslots, sl = idx % nslots;
  out[(size_t)sl * world + rk] = in[(size_t)rk * 8 + sl];
}

__global__ void k_scale(Fr* __restrict__ a, size_t n, const Fr* __restrict__ s) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = a[i] * (*s);
}

}  // namespace qg

// ---------------------------------------------------------------- host driver
namespace qg {

void eq_table_device(qg_ctx* ctx, const Fr* d_z, uint32_t nvars, Fr* d_out) {
  QgTimed tm(ctx, "eq_table");
  const size_t n = (size_t)1 << nvars;
  if (nvars <= 12) {
    hipLaunchKernelGGL(k_eq_small, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_z, 0u,
                       nvars, d_out);
    QG_LAUNCH_CHECK();
    return;
  }
  const uint32_t lb = nvars / 2, hb = nvars - lb;
  Fr* low = ctx->scratch_as<Fr>("eq_low", (size_t)1 << lb);
  Fr* high = ctx->scratch_as<Fr>("eq_high", (size_t)1 << hb);
  hipLaunchKernelGGL(k_eq_small, dim3(div_up((size_t)1 << lb, 256)), dim3(256), 0, ctx->stream,
                     d_z, 0u, lb, low);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eq_small, dim3(div_up((size_t)1 << hb, 256)), dim3(256), 0, ctx->stream,
                     d_z, lb, hb, high);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_eq_combine, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, low, high, lb,
                     n, d_out);
  QG_LAUNCH_CHECK();
}

struct SumcheckResult {
  std::vector<uint64_t> coeffs;  // nvars * width * 4
  std::vector<uint32_t> lens;
  std::vector<Fr> point;
  Fr evaluation;
};

template <int K, int NPMAX>
static void run_rounds(qg_ctx* ctx, uint32_t nvars, const std::vector<const Fr*>& src,
                       const SopDev* d_sp, uint32_t nslots, RoundOut ro, Fr* d_final,
                       Fr* d_eval) {
  const size_t N = (size_t)1 << nvars;
  // ping-pong scratch: X holds N/2 per slot, Y holds N/4 per slot
  Fr* X = ctx->scratch_as<Fr>("sc_x", std::max<size_t>(1, (N / 2) * nslots));
  Fr* Y = ctx->scratch_as<Fr>("sc_y", std::max<size_t>(1, (N / 4) * nslots));
  Fr* partial = ctx->scratch_as<Fr>("sc_partial", (size_t)SC_MAX_BLOCKS * NPMAX);
  TablePtrs cur{};
  for (uint32_t i = 0; i < 8; i++) cur.src[i] = i < nslots ? src[i] : nullptr;
  auto bufs = [&](Fr* base, size_t per) {
    TablePtrs t{};
    for (uint32_t i = 0; i < 8; i++) t.dst[i] = i < nslots ? base + per * i : nullptr;
    return t;
  };
  TablePtrs tX = bufs(X, N / 2), tY = bufs(Y, std::max<size_t>(1, N / 4));
  int fold = 0;
  uint32_t j = 0;
  int parity = 0;  // next destination: 0 -> X, 1 -> Y
  {
    QgTimed tm(ctx, "sumcheck_round");
    for (; j < nvars; j++) {
      const size_t table = N >> j;  // logical size before this round's fold... after fold
      // size of the tables this round evaluates: N >> j
      if (table <= ((size_t)1 << TAIL_LOG)) break;
      const size_t npairs = table / 2;
      unsigned blocks = (unsigned)std::min<size_t>(SC_MAX_BLOCKS, div_up(npairs, SC_BLOCK));
      TablePtrs tp = cur;
      if (fold) {
        const TablePtrs& d = parity ? tY : tX;
        for (int i = 0; i < 8; i++) tp.dst[i] = d.dst[i];
      }
      hipLaunchKernelGGL((k_sc_round<K, NPMAX>), dim3(blocks), dim3(SC_BLOCK), 0, ctx->stream, tp,
                         d_sp, npairs, fold, fold ? ro.chal + (j - 1) : ro.chal, partial);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL((k_sc_finish<NPMAX>), dim3(1), dim3(SC_BLOCK), 0, ctx->stream, d_sp,
                         partial, blocks, ro, j);
      QG_LAUNCH_CHECK();
      if (fold) {
        for (int i = 0; i < 8; i++) cur.src[i] = tp.dst[i];
        parity ^= 1;
      }
      fold = 1;
    }
  }
  {
    QgTimed tm(ctx, "sumcheck_tail");
    // Tail destinations.  k_sc_tail writes round j0's fold into t0.dst, then
    // alternates bufA, bufB, bufA, ...  Capacities: X >= N/2, Y >= N/4.
    //  j0 == 0: round 0 does not fold; round 1 writes N/2 -> X, round 2 -> Y, ...
    //  j0 >= 1: round j0 writes N>>j0 into the buffer not holding cur.src
    //           (X when parity == 0, j0 >= 1; Y when parity == 1, j0 >= 2).
    TablePtrs t0 = cur, bufA, bufB;
    if (j == 0) {
      bufA = tX;
      bufB = tY;
    } else {
      const TablePtrs& a = parity ? tY : tX;
      const TablePtrs& b = parity ? tX : tY;
      for (int i = 0; i < 8; i++) t0.dst[i] = a.dst[i];
      bufA = b;
      bufB = a;
    }
    hipLaunchKernelGGL((k_sc_tail<K, NPMAX>), dim3(1), dim3(SC_BLOCK), 0, ctx->stream, t0, bufA,
                       bufB, d_sp, nvars, j, fold, ro, d_final, d_eval);
    QG_LAUNCH_CHECK();
  }
}

// Sharded rounds: this rank holds the block of every table whose
// high log2(world) index bits equal its rank.  Rounds 0..m-1 (m = local bits)
// pair local entries only: one allgather of the (d+1) round sums per round, then
// every rank runs the identical device transcript.  The last log2(world) rounds
// run redundantly on the allgathered single values.
template <int K, int NPMAX>
static void run_rounds_dist(qg_ctx* ctx, uint32_t nvars, const std::vector<const Fr*>& src,
                            const SopDev* d_sp, uint32_t nslots, RoundOut ro, Fr* d_final,
                            Fr* d_eval) {
  const uint32_t world = (uint32_t)ctx->world;
  uint32_t lw = 0;
  while ((1u << lw) < world) lw++;
  QG_CHECK((1u << lw) == world, QG_ERR_INVALID, "sharded sumcheck needs a power-of-two world");
  QG_CHECK(nvars > lw, QG_ERR_INVALID, "sharded sumcheck needs nvars > log2(world)");
  const uint32_t m = nvars - lw;
  const size_t NL = (size_t)1 << m;
  Fr* X = ctx->scratch_as<Fr>("sc_x", std::max<size_t>(1, (NL / 2) * std::max(nslots, 1u)));
  Fr* Y = ctx->scratch_as<Fr>("sc_y", std::max<size_t>(1, (NL / 4) * std::max(nslots, 1u)));
  Fr* partial = ctx->scratch_as<Fr>("sc_partial", (size_t)SC_MAX_BLOCKS * NPMAX);
  Fr* loc = ctx->scratch_as<Fr>("sc_loc", NPMAX);
  Fr* all = ctx->scratch_as<Fr>("sc_all", (size_t)world * NPMAX);
  Fr* last = ctx->scratch_as<Fr>("sc_last", 8);
  Fr* graw = ctx->scratch_as<Fr>("sc_graw", (size_t)world * 8);
  Fr* gt = ctx->scratch_as<Fr>("sc_gt", (size_t)world * 8);
  Fr* gA = ctx->scratch_as<Fr>("sc_gA", (size_t)world * 8);
  Fr* gB = ctx->scratch_as<Fr>("sc_gB", (size_t)world * 8);
  TablePtrs cur{};
  for (uint32_t i = 0; i < 8; i++) cur.src[i] = i < nslots ? src[i] : nullptr;
  auto bufs = [&](Fr* base, size_t per) {
    TablePtrs t{};
    for (uint32_t i = 0; i < 8; i++) t.dst[i] = i < nslots ? base + per * i : nullptr;
    return t;
  };
  TablePtrs tX = bufs(X, NL / 2), tY = bufs(Y, std::max<size_t>(1, NL / 4));
  int fold = 0, parity = 0;
  {
    QgTimed tm(ctx, "sumcheck_round");
    for (uint32_t j = 0; j < m; j++) {
      const size_t npairs = (NL >> j) / 2;
      const unsigned blocks = (unsigned)std::min<size_t>(SC_MAX_BLOCKS, div_up(npairs, SC_BLOCK));
      TablePtrs tp = cur;
      if (fold) {
        const TablePtrs& d = parity ? tY : tX;
        for (int i = 0; i < 8; i++) tp.dst[i] = d.dst[i];
      }
      hipLaunchKernelGGL((k_sc_round<K, NPMAX>), dim3(blocks), dim3(SC_BLOCK), 0, ctx->stream, tp,
                         d_sp, npairs, fold, fold ? ro.chal + (j - 1) : ro.chal, partial);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL((k_sc_local_sum<NPMAX>), dim3(1), dim3(SC_BLOCK), 0, ctx->stream, d_sp,
                         partial, blocks, loc);
      QG_LAUNCH_CHECK();
      comm_allgather_bytes(ctx, loc, all, sizeof(Fr) * NPMAX);
      hipLaunchKernelGGL((k_sc_finish<NPMAX>), dim3(1), dim3(SC_BLOCK), 0, ctx->stream, d_sp, all,
                         world, ro, j);
      QG_LAUNCH_CHECK();
      if (fold) {
        for (int i = 0; i < 8; i++) cur.src[i] = tp.dst[i];
        parity ^= 1;
      }
      fold = 1;
    }
  }
  {
    QgTimed tm(ctx, "sumcheck_tail");
    // local tables have 2 entries (folded through r_{m-2}); fold with r_{m-1}
    if (nslots) {
      hipLaunchKernelGGL(k_sc_fold_last, dim3(1), dim3(64), 0, ctx->stream, cur, nslots,
                         ro.chal + (m - 1), last);
      QG_LAUNCH_CHECK();
    }
    comm_allgather_bytes(ctx, last, graw, sizeof(Fr) * 8);
    if (nslots) {
      hipLaunchKernelGGL(k_sc_transpose, dim3(div_up((size_t)world * nslots, 64)), dim3(64), 0,
                         ctx->stream, graw, world, nslots, gt);
      QG_LAUNCH_CHECK();
    }
    TablePtrs t0{}, bufA{}, bufB{};
    for (uint32_t i = 0; i < 8; i++) {
      t0.src[i] = i < nslots ? gt + (size_t)world * i : nullptr;
      bufA.dst[i] = i < nslots ? gA + (size_t)world * i : nullptr;
      bufB.dst[i] = i < nslots ? gB + (size_t)world * i : nullptr;
    }
    hipLaunchKernelGGL((k_sc_tail<K, NPMAX>), dim3(1), dim3(SC_BLOCK), 0, ctx->stream, t0, bufA,
                       bufB, d_sp, nvars, m, 0, ro, d_final, d_eval);
    QG_LAUNCH_CHECK();
  }
}

template <int K, int NPMAX>
static void run_rounds_any(qg_ctx* ctx, uint32_t nvars, const std::vector<const Fr*>& src,
                           const SopDev* d_sp, uint32_t nslots, RoundOut ro, Fr* d_final,
                           Fr* d_eval) {
  if (ctx->world > 1) run_rounds_dist<K, NPMAX>(ctx, nvars, src, d_sp, nslots, ro, d_final, d_eval);
  else run_rounds<K, NPMAX>(ctx, nvars, src, d_sp, nslots, ro, d_final, d_eval);
}

static void sumcheck_run(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                         const std::vector<const Fr*>& d_tables, const qg_expr_op* prog,
                         size_t prog_len, const uint64_t* consts, size_t nconsts,
                         const uint64_t claimed_sum[4], uint8_t state[32], uint64_t* round_coeffs,
                         uint32_t* round_lens, uint64_t* point, uint64_t evaluation[4]) {
  QG_CHECK(nvars >= 1 && nvars <= 40, QG_ERR_INVALID, "nvars out of range");
  const uint32_t width = expr_degree(prog, prog_len) + 1;
  SopProgram sp = compile_program(prog, prog_len, consts, nconsts, ntables);
  QG_CHECK(sp.mono_len.size() <= 256 && sp.fac.size() <= 1024, QG_ERR_UNSUPPORTED,
           "expression too large");
  QG_CHECK(sp.used.size() <= 8, QG_ERR_UNSUPPORTED, "expression uses more than 8 tables");
  QG_CHECK(sp.degree <= 15, QG_ERR_UNSUPPORTED, "expression degree above 15");
  const uint32_t np = sp.degree + 1;
  QG_CHECK(np <= width, QG_ERR_ASSERT, "degree bookkeeping");

  // transcript: append num_vars (usize) and claimed_sum (sumcheck.rs:35-36)
  uint8_t st[32];
  memcpy(st, state, 32);
  uint8_t b8[8], b32[32];
  u64_to_bytes(nvars, b8);
  transcript_append(st, b8, 8);
  fr_to_bytes(fr_import(claimed_sum), b32);
  transcript_append(st, b32, 32);

  SopDev* h_sp = new SopDev();
  memset(h_sp, 0, sizeof(SopDev));
  h_sp->nmono = (uint32_t)sp.mono_len.size();
  h_sp->nslots = (uint32_t)sp.used.size();
  h_sp->np = np;
  for (size_t m = 0; m < sp.mono_len.size(); m++) {
    h_sp->mono_len[m] = sp.mono_len[m];
    h_sp->is_one[m] = sp.is_one[m];
    h_sp->coeff[m] = sp.coeff[m];
  }
  for (size_t f = 0; f < sp.fac.size(); f++) h_sp->fac[f] = (uint8_t)sp.fac[f];
  build_vinv(np, h_sp->vinv);

  SopDev* d_sp = ctx->scratch_as<SopDev>("sc_prog", 1);
  uint32_t* d_state = ctx->scratch_as<uint32_t>("sc_state", 8);
  Fr* d_chal = ctx->scratch_as<Fr>("sc_chal", nvars);
  Fr* d_coeffs = ctx->scratch_as<Fr>("sc_coeffs", (size_t)nvars * width);
  uint32_t* d_lens = ctx->scratch_as<uint32_t>("sc_lens", nvars);
  Fr* d_final = ctx->scratch_as<Fr>("sc_final", 9);
  QG_HIP(hipMemcpyAsync(d_sp, h_sp, sizeof(SopDev), hipMemcpyHostToDevice, ctx->stream));
  QG_HIP(hipMemcpyAsync(d_state, st, 32, hipMemcpyHostToDevice, ctx->stream));

  std::vector<const Fr*> src;
  for (uint32_t u : sp.used) src.push_back(d_tables[u]);
  RoundOut ro{d_state, d_chal, d_coeffs, d_lens, width};
  Fr* d_eval = d_final + 8;

  if (sp.used.empty()) {
    // constant expression: every table slot unused; evaluate with K = 1 and a dummy slot
    src.push_back(d_tables.empty() ? d_chal : d_tables[0]);
  }
  const uint32_t nslots_launch = (uint32_t)sp.used.size();
  // (with no used slots, nslots = 0 and loads are skipped)
  if (np <= 4) {
    if (src.size() <= 4) run_rounds_any<4, 4>(ctx, nvars, src, d_sp, nslots_launch, ro, d_final, d_eval);
    else run_rounds_any<8, 4>(ctx, nvars, src, d_sp, nslots_launch, ro, d_final, d_eval);
  } else if (np <= 8) {
    if (src.size() <= 4) run_rounds_any<4, 8>(ctx, nvars, src, d_sp, nslots_launch, ro, d_final, d_eval);
    else run_rounds_any<8, 8>(ctx, nvars, src, d_sp, nslots_launch, ro, d_final, d_eval);
  } else {
    run_rounds_any<8, 16>(ctx, nvars, src, d_sp, nslots_launch, ro, d_final, d_eval);
  }

  std::vector<Fr> h_coeffs((size_t)nvars * width), h_chal(nvars);
  Fr h_eval;
  QG_HIP(hipMemcpyAsync(h_coeffs.data(), d_coeffs, sizeof(Fr) * h_coeffs.size(),
                        hipMemcpyDeviceToHost, ctx->stream));
  QG_HIP(hipMemcpyAsync(round_lens, d_lens, sizeof(uint32_t) * nvars, hipMemcpyDeviceToHost,
                        ctx->stream));
  QG_HIP(hipMemcpyAsync(h_chal.data(), d_chal, sizeof(Fr) * nvars, hipMemcpyDeviceToHost,
                        ctx->stream));
  QG_HIP(hipMemcpyAsync(&h_eval, d_eval, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  QG_HIP(hipMemcpyAsync(state, d_state, 32, hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  delete h_sp;
  for (size_t i = 0; i < h_coeffs.size(); i++) fr_export(h_coeffs[i], round_coeffs + 4 * i);
  for (uint32_t i = 0; i < nvars; i++) fr_export(h_chal[i], point + 4 * i);
  fr_export(h_eval, evaluation);
}

// entries per table held by this rank: 2^nvars, or 2^(nvars - log2(world)) when
// the tables are sharded over an attached communicator
static size_t local_table_size(const qg_ctx* ctx, uint32_t nvars) {
  uint32_t lw = 0;
  while ((1 << lw) < ctx->world) lw++;
  QG_CHECK((1 << lw) == ctx->world, QG_ERR_INVALID, "world size must be a power of two");
  QG_CHECK(nvars > lw, QG_ERR_INVALID, "nvars must exceed log2(world)");
  return (size_t)1 << (nvars - lw);
}

static std::vector<const Fr*> upload_tables(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                                            const uint64_t* const* tables) {
  const size_t N = local_table_size(ctx, nvars);
  Fr* d = ctx->scratch_as<Fr>("sc_in", std::max<size_t>(1, N * ntables));
  std::vector<const Fr*> out;
  for (uint32_t i = 0; i < ntables; i++) {
    QG_CHECK(tables[i] != nullptr, QG_ERR_INVALID, "null table");
    fr_upload(ctx, d + N * i, tables[i], N);
    out.push_back(d + N * i);
  }
  return out;
}

// zero-check driver: draw z, eq table, sumcheck of h * eq with sum 0
static void zerocheck_run(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                          std::vector<const Fr*> d_tables, const qg_expr_op* prog, size_t prog_len,
                          const uint64_t* consts, size_t nconsts, uint8_t state[32],
                          uint64_t* round_coeffs, uint32_t* round_lens, uint64_t* point,
                          uint64_t evaluation[4], uint64_t* eq_out) {
  QG_CHECK(nvars >= 1 && nvars <= 40, QG_ERR_INVALID, "nvars out of range");
  std::vector<Fr> z(nvars);
  for (uint32_t i = 0; i < nvars; i++) z[i] = transcript_draw_fr(state);  // zerocheck.rs:20-22
  const size_t N = local_table_size(ctx, nvars);
  uint32_t m = 0;
  while (((size_t)1 << m) < N) m++;
  Fr* d_z = ctx->scratch_as<Fr>("zc_z", nvars);
  Fr* d_eq = ctx->scratch_as<Fr>("zc_eq", N);
  QG_HIP(hipMemcpyAsync(d_z, z.data(), sizeof(Fr) * nvars, hipMemcpyHostToDevice, ctx->stream));
  eq_table_device(ctx, d_z, m, d_eq);
  if (ctx->world > 1) {
    // this rank's block: the high index bits are the rank (eq_eval.rs bit j <-> z_j)
    Fr f = Fr::one();
    for (uint32_t j = m; j < nvars; j++)
      f = f * ((((uint32_t)ctx->rank >> (j - m)) & 1u) ? z[j] : Fr::one() - z[j]);
    Fr* d_f = ctx->scratch_as<Fr>("zc_f", 1);
    QG_HIP(hipMemcpyAsync(d_f, &f, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_scale, dim3(div_up(N, 256)), dim3(256), 0, ctx->stream, d_eq, N, d_f);
    QG_LAUNCH_CHECK();
    ctx->sync();  // f lives on the host stack
  }
  if (eq_out) fr_download(ctx, eq_out, d_eq, N);
  d_tables.push_back(d_eq);
  std::vector<qg_expr_op> p2(prog, prog + prog_len);
  p2.push_back({QG_OP_INPUT, ntables});
  p2.push_back({QG_OP_MUL, 0});
  uint64_t zero[4] = {0, 0, 0, 0};
  sumcheck_run(ctx, nvars, ntables + 1, d_tables, p2.data(), p2.size(), consts, nconsts, zero,
               state, round_coeffs, round_lens, point, evaluation);
  // claim / eq(z, point)   (zerocheck.rs:34-40)
  Fr e = Fr::one();
  for (uint32_t i = 0; i < nvars; i++) {
    Fr x = fr_import(point + 4 * i);
    e = e * (x * z[i] + (Fr::one() - x) * (Fr::one() - z[i]));
  }
  Fr ev = fr_import(evaluation) * finv(e);
  fr_export(ev, evaluation);
}

}  // namespace qg

extern "C" {

int qg_expr_degree(const qg_expr_op* prog, size_t prog_len, uint32_t* out_degree) {
  if (!prog || !out_degree) return QG_ERR_INVALID;
  return qg_guard(nullptr, [&] { *out_degree = expr_degree(prog, prog_len); });
}

int qg_eq_table(qg_ctx* ctx, const uint64_t* point, size_t nvars, uint64_t* out) {
  if (!ctx || (!point && nvars) || !out || nvars > 34) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    const size_t N = (size_t)1 << nvars;
    Fr* d_z = ctx->scratch_as<Fr>("eq_z", nvars ? nvars : 1);
    Fr* d_out = ctx->scratch_as<Fr>("eq_out", N);
    fr_upload(ctx, d_z, point, nvars);
    eq_table_device(ctx, d_z, (uint32_t)nvars, d_out);
    fr_download(ctx, out, d_out, N);
    ctx->sync();
  });
}

int qg_sumcheck_prove(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                      const uint64_t* const* tables, const qg_expr_op* prog, size_t prog_len,
                      const uint64_t* consts, size_t nconsts, const uint64_t claimed_sum[4],
                      uint8_t state[32], uint64_t* round_coeffs, uint32_t* round_lens,
                      uint64_t* point, uint64_t evaluation[4]) {
  if (!ctx || (!tables && ntables) || !prog || !claimed_sum || !state || !round_coeffs ||
      !round_lens || !point || !evaluation || (!consts && nconsts))
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars >= 1 && nvars <= 34, QG_ERR_INVALID, "nvars out of range");
    QG_HIP(hipSetDevice(ctx->device));
    auto d = upload_tables(ctx, nvars, ntables, tables);
    sumcheck_run(ctx, nvars, ntables, d, prog, prog_len, consts, nconsts, claimed_sum, state,
                 round_coeffs, round_lens, point, evaluation);
  });
}

int qg_sumcheck_prove_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                          const qg_buf* const* tables, const qg_expr_op* prog, size_t prog_len,
                          const uint64_t* consts, size_t nconsts, const uint64_t claimed_sum[4],
                          uint8_t state[32], uint64_t* round_coeffs, uint32_t* round_lens,
                          uint64_t* point, uint64_t evaluation[4]) {
  if (!ctx || (!tables && ntables) || !prog || !claimed_sum || !state || !round_coeffs ||
      !round_lens || !point || !evaluation || (!consts && nconsts))
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars >= 1 && nvars <= 34, QG_ERR_INVALID, "nvars out of range");
    QG_HIP(hipSetDevice(ctx->device));
    std::vector<const Fr*> d;
    for (uint32_t i = 0; i < ntables; i++) {
      QG_CHECK(tables[i] && tables[i]->n >= local_table_size(ctx, nvars), QG_ERR_INVALID,
               "device table shorter than its (local) hypercube size");
      d.push_back(tables[i]->d);
    }
    sumcheck_run(ctx, nvars, ntables, d, prog, prog_len, consts, nconsts, claimed_sum, state,
                 round_coeffs, round_lens, point, evaluation);
  });
}

int qg_zerocheck_prove(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                       const uint64_t* const* tables, const qg_expr_op* prog, size_t prog_len,
                       const uint64_t* consts, size_t nconsts, uint8_t state[32],
                       uint64_t* round_coeffs, uint32_t* round_lens, uint64_t* point,
                       uint64_t evaluation[4], uint64_t* eq_out) {
  if (!ctx || (!tables && ntables) || !prog || !state || !round_coeffs || !round_lens || !point ||
      !evaluation || (!consts && nconsts))
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars >= 1 && nvars <= 34, QG_ERR_INVALID, "nvars out of range");
    QG_HIP(hipSetDevice(ctx->device));
    auto d = upload_tables(ctx, nvars, ntables, tables);
    zerocheck_run(ctx, nvars, ntables, d, prog, prog_len, consts, nconsts, state, round_coeffs,
                  round_lens, point, evaluation, eq_out);
  });
}

int qg_zerocheck_prove_dev(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                           const qg_buf* const* tables, const qg_expr_op* prog, size_t prog_len,
                           const uint64_t* consts, size_t nconsts, uint8_t state[32],
                           uint64_t* round_coeffs, uint32_t* round_lens, uint64_t* point,
                           uint64_t evaluation[4]) {
  if (!ctx || (!tables && ntables) || !prog || !state || !round_coeffs || !round_lens || !point ||
      !evaluation || (!consts && nconsts))
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars >= 1 && nvars <= 34, QG_ERR_INVALID, "nvars out of range");
    QG_HIP(hipSetDevice(ctx->device));
    std::vector<const Fr*> d;
    for (uint32_t i = 0; i < ntables; i++) {
      QG_CHECK(tables[i] && tables[i]->n >= local_table_size(ctx, nvars), QG_ERR_INVALID,
               "device table shorter than its (local) hypercube size");
      d.push_back(tables[i]->d);
    }
    zerocheck_run(ctx, nvars, ntables, d, prog, prog_len, consts, nconsts, state, round_coeffs,
                  round_lens, point, evaluation, nullptr);
  });
}

}  // extern "C"
