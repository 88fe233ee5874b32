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
//  * Once a table has <= 2^PERS_LOG entries the remaining rounds run inside one
//    workgroup (fold + evaluate + transcript per round, synchronized by
//    barriers), removing 2 launches per round.
#include <stddef.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "blake3.h"
#include "common.h"
#include "expr.h"
#include "field29.h"

using namespace qg;

namespace qg {

// Phase timestamps (s_memrealtime, 100 MHz) for latency work: build with
// -DQG_SC_TRACE (make trace) and read them with qg_debug_sc_trace.
#ifdef QG_SC_TRACE
__device__ unsigned long long g_sc_trace[2048 + 4 * 1536];
#define SC_TR(idx)                                                   \
  do {                                                               \
    if (threadIdx.x == 0 && (idx) < 2048) g_sc_trace[idx] = wall_clock64(); \
  } while (0)
// per-block (start, sweep end, CU id) of big rounds 0..3, blocks < 512
#define SC_TB(j, k)                                                                   \
  do {                                                                                \
    if (threadIdx.x == 0 && (j) < 4 && blockIdx.x < 512) {                            \
      g_sc_trace[2048 + (j) * 1536 + 3 * blockIdx.x + (k)] = wall_clock64();          \
      if ((k) == 0) g_sc_trace[2048 + (j) * 1536 + 3 * blockIdx.x + 2] = __smid();    \
    }                                                                                 \
  } while (0)
// per-wave (sweep end, HW_ID) of big rounds 0..3, blocks < 512, waves < 8
__device__ unsigned long long g_sc_wtrace[4 * 512 * 8 * 2];
#define SC_TW(j)                                                                          \
  do {                                                                                    \
    if ((threadIdx.x & 63) == 0 && (j) < 4 && blockIdx.x < 512 && (threadIdx.x >> 6) < 8) { \
      const size_t o = (((size_t)(j) * 512 + blockIdx.x) * 8 + (threadIdx.x >> 6)) * 2;    \
      g_sc_wtrace[o] = wall_clock64();                                                    \
      g_sc_wtrace[o + 1] = __builtin_amdgcn_s_getreg(63492) /* HW_REG_HW_ID */          \
                           | ((unsigned long long)__builtin_amdgcn_s_getreg(6164) << 32); /* XCC_ID */ \
    }                                                                                     \
  } while (0)
#else
#define SC_TW(j) \
  do {           \
  } while (0)
#define SC_TR(idx) \
  do {             \
  } while (0)
#define SC_TB(j, k) \
  do {              \
  } while (0)
#endif

static constexpr int SC_BLOCK = 256;
static constexpr int SC_MAX_BLOCKS = 2048;  // partial-sum capacity (blocks per big round)

// blocks of a big round: ~3 resident blocks per CU, each striding over many
// pair groups (measured on MI355X at 2^20 vars: 768 blocks 0.764 ms vs 2048
// blocks 0.798 ms; QG_SC_BLOCKS overrides, for tuning)
static unsigned sc_round_blocks(qg_ctx* ctx, size_t npairs) {
  static int ov = [] {
    const char* e = getenv("QG_SC_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  size_t cap = ov > 0 ? (size_t)ov : (size_t)3 * ctx->num_cus();
  cap = std::min<size_t>(cap, SC_MAX_BLOCKS);
  return (unsigned)std::max<size_t>(1, std::min<size_t>(cap, div_up(npairs, SC_BLOCK)));
}
// QG_SC_STAGED=1 selects the LDS-staged round kernels (k_sc_round) for the big
// rounds on one GPU, for A/B runs
static bool sc_use_staged() {
  static const bool v = getenv("QG_SC_STAGED") != nullptr;
  return v;
}
static constexpr int PERS_LOG = 16;     // tables of <= 2^16 entries: rounds run in one persistent launch

// device-side program image.  The header and byte arrays are copied into LDS
// by every block (one parallel load, no dependent scalar-cache misses on the
// evaluation path), followed by the 29-bit-limb constants.
//
// Arithmetic scale (field29.h): table entries are arkworks Montgomery values
// (x * 2^256) re-limbed to 9 x 29 bits; mul29 multiplies by 2^-261.  A product
// of d entries therefore carries 2^(256 - 5(d-1)).  The round sums are kept at
// S = 2^(256 - 5(dmax-1)): a degree-dmax monomial with coefficient 1 is added
// as is; any other monomial is multiplied by c * 2^(261 - 5(dmax-d)); a
// constant term is stored as c * S.  The interpolation constants undo S.
static constexpr int SOP_MAXM = 256, SOP_MAXF = 1024;
static constexpr uint32_t SOP_HDR_WORDS = (16 + 2 * SOP_MAXM + SOP_MAXF) / 4;

struct SopDev {
  uint32_t nmono, nslots, np, nfac;
  uint8_t mono_len[SOP_MAXM];
  uint8_t skip29[SOP_MAXM];  // 1: product already at scale S (no multiply)
  uint8_t fac[SOP_MAXF];
  L9 c29[SOP_MAXM];          // per-monomial multiplier (or constant term), plain integer
  L9 vm29[16 * 16];          // interpolation -> Montgomery coefficients (R = 2^256)
  L9 vc29[16 * 16];          // interpolation -> canonical coefficients (transcript bytes)
  L9 t29[16];                // t * 2^261 mod p (evaluation-point offsets, NP > 4)
  L9 cr29[4];                // 2^522, 2^778 (-> r * 2^261); 2^517, 2^773 (-> r * 2^256)
  Fr coeff[SOP_MAXM];        // Montgomery coefficients (final claim on the 32-bit path)
  uint8_t is_one[SOP_MAXM];  // (final claim)
  L9 cs29;                   // 2^(517 - e): canonical value -> scale S (the round claim)
};
static_assert(offsetof(SopDev, c29) == SOP_HDR_WORDS * 4, "SopDev layout");

// program header passed by value (no dependent loads before the LDS copy)
struct SopHdr {
  uint32_t nmono, nslots, np, pad;  // pad: SOP_* flags
};
// the expression is the product of every used slot once, in slot order, with
// coefficient 1 (h = g1 g2 ... gk): evaluated without slot picks
static constexpr uint32_t SOP_PURE = 1;

using R29 = F29<FrP>;

template <int NP>
struct SopLds {
  uint32_t w[SOP_HDR_WORDS];
  R29 c29[SOP_MAXM];
  R29 vm[NP * NP];
  R29 vc[NP * NP];
  R29 t29[NP];
  R29 cr[4];
  QG_DEV uint32_t nmono() const { return w[0]; }
  QG_DEV uint32_t mono_len(uint32_t m) const { return ((const uint8_t*)w)[16 + m]; }
  QG_DEV uint32_t skip(uint32_t m) const { return ((const uint8_t*)w)[16 + SOP_MAXM + m]; }
  QG_DEV uint32_t fac(uint32_t f) const { return ((const uint8_t*)w)[16 + 2 * SOP_MAXM + f]; }
};

template <int NP>
QG_DEV void sop_load(SopLds<NP>& s, const SopDev* __restrict__ g, const SopHdr& h, bool vinv) {
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  const uint32_t* gw = reinterpret_cast<const uint32_t*>(g);
  for (uint32_t i = tid; i < SOP_HDR_WORDS; i += nt) s.w[i] = gw[i];
  const uint32_t* gc = reinterpret_cast<const uint32_t*>(g->c29);
  uint32_t* lc = reinterpret_cast<uint32_t*>(s.c29);
  for (uint32_t i = tid; i < h.nmono * 9; i += nt) lc[i] = gc[i];
  for (uint32_t i = tid; i < NP * 9; i += nt)
    reinterpret_cast<uint32_t*>(s.t29)[i] = reinterpret_cast<const uint32_t*>(g->t29)[i];
  for (uint32_t i = tid; i < 4 * 9; i += nt)
    reinterpret_cast<uint32_t*>(s.cr)[i] = reinterpret_cast<const uint32_t*>(g->cr29)[i];
  if (vinv) {
    for (uint32_t i = tid; i < h.np * h.np * 9; i += nt) {
      const uint32_t e = i / 9, k = i % 9, t = e / h.np, u = e % h.np;
      s.vm[t * NP + u].l[k] = g->vm29[t * 16 + u].v[k];
      s.vc[t * NP + u].l[k] = g->vc29[t * 16 + u].v[k];
    }
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

// h(values) on the 32-bit path (final claim): Montgomery coefficients from HBM
template <int K>
QG_DEV Fr sop_eval_final(const SopDev* __restrict__ g, uint32_t nmono, const Fr (&val)[K]) {
  Fr acc = Fr::zero();
  uint32_t f = 0;
  for (uint32_t m = 0; m < nmono; m++) {
    const uint32_t len = g->mono_len[m];
    Fr prod;
    if (len == 0) {
      prod = g->coeff[m];
    } else {
      prod = sel<K>(val, g->fac[f]);
      for (uint32_t q = 1; q < len; q++) prod = prod * sel<K>(val, g->fac[f + q]);
      if (!g->is_one[m]) prod = prod * g->coeff[m];
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

// ---------------------------------------------------------------- in-launch hand-offs
// Data handed between workgroups INSIDE one launch (partial rows, the
// persistent tail's folded tables, the transcript state of the big rounds) is
// stored write-through and loaded L1-bypassing: agent-scope relaxed atomics on
// GLOBAL pointers lower to `global_store/load ... sc1` (MI355X_MICROARCH.md
// "Valid forms", first row: one lane signals by an agent-scope atomic after
// every storing wave's vmcnt(0) wait and a workgroup barrier; the consumer
// polls that counter with an sc1 load and loads every handed-off byte with sc1
// loads).  No release fence, so no `buffer_wbl2` write-back of the XCD L2's
// dirty table lines on the critical path.
typedef __attribute__((address_space(1))) uint64_t gu64;
typedef __attribute__((address_space(1))) uint32_t gu32;

QG_DEV Fr ld_sc1(const Fr* p) {
  gu64* q = (gu64*)(const_cast<Fr*>(p));
  Fr r;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t v = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    r.v[2 * i] = (uint32_t)v;
    r.v[2 * i + 1] = (uint32_t)(v >> 32);
  }
  return r;
}
QG_DEV void st_sc1(Fr* p, const Fr& x) {
  gu64* q = (gu64*)p;
#pragma unroll
  for (int i = 0; i < 4; i++)
    __hip_atomic_store(q + i, (uint64_t)x.v[2 * i] | ((uint64_t)x.v[2 * i + 1] << 32),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
QG_DEV uint32_t ld_sc1_u32(const uint32_t* p) {
  return __hip_atomic_load((gu32*)(const_cast<uint32_t*>(p)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}
QG_DEV void st_sc1_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// every storing wave drains its sc1 stores (inline asm: the compiler cannot drop it)
QG_DEV void drain_stores() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

QG_DEV Fr shfl_xor_fr(const Fr& a, int m) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __shfl_xor(a.v[i], m, 64);
  return r;
}

// lazy value < 6p -> normalized, < 2p
QG_DEV R29 red6p(const R29& a) {
  return condsub29<FrP>(condsub29<FrP>(normfull29<FrP>(a), l9_mul_small(F29P<FrP>::P, 4)),
                        F29P<FrP>::P2);
}

// x < 2^256 as 8 x 32 words, reduced modulo p below 2p (values here are < 3p)
QG_DEV Fr lt_p(const Fr& x) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = x.v[i];
  reduce_once<FrP>(t);
  reduce_once<FrP>(t);
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = t[i];
  return r;
}

// ---------------------------------------------------------------------------
// Work layout of a round.  A block handles PB = BLOCK / NP pairs per step:
//   phase F: items (slot, pair, half) — fold (x0 + r (x1 - x0)) or copy one
//            entry of the next table into LDS (and HBM when folding);
//   phase E: thread (pair = tid / NP, point t = tid % NP) evaluates h at
//            lo + t (hi - lo) and accumulates its own point's sum.
// Every thread carries one field accumulator, so registers stay low (high
// occupancy on the large rounds) and the dependent chain per round is one
// fold multiply plus deg-1 product multiplies (low latency on the small ones).
// All arithmetic is 29-bit-limb (field29.h); folded tables are stored < 2p.
// ---------------------------------------------------------------------------
template <int K, int NP, int BLOCK>
struct RoundLds {
  R29 F[K * (BLOCK / NP) * 2];  // [slot][pair][half]
  const Fr* src[8];
  Fr* dst[8];
};

template <int K, int NP, int BLOCK>
QG_DEV void round_sweep(RoundLds<K, NP, BLOCK>& L, const SopLds<NP>& sp, const SopHdr& h,
                        size_t npairs, bool fold, const R29& r, size_t base0, size_t stride,
                        R29& acc) {
  constexpr uint32_t PB = BLOCK / NP;
  const uint32_t tid = threadIdx.x, t = tid % NP, pl = tid / NP;
  const uint32_t nitems = h.nslots * PB * 2;
  for (size_t base = base0; base < npairs; base += stride) {
    for (uint32_t it = tid; it < nitems; it += BLOCK) {
      const uint32_t s = it / (PB * 2), e = it % (PB * 2);
      const size_t p = base + (e >> 1);
      R29 v = R29::zero();
      if (p < npairs) {
        if (fold) {
          const Fr* src = L.src[s] + 4 * p + 2 * (e & 1);
          const R29 x0 = to29(src[0]), x1 = to29(src[1]);
          // x0 + r (x1 - x0): x1 - x0 + 4p (lazy) times r (< 2p) -> < 2p; + x0 -> < 4p
          v = red2p29<FrP>(add29(x0, mul29(sub29(x1, x0), r)));
          L.dst[s][2 * p + (e & 1)] = from29(v);
        } else {
          v = to29(L.src[s][2 * p + (e & 1)]);
        }
      }
      L.F[s * PB * 2 + e] = v;
    }
    __syncthreads();
    if (t < h.np && base + pl < npairs) {
      R29 sum = R29::zero();
      uint32_t f = 0;
      for (uint32_t m = 0; m < h.nmono; m++) {
        const uint32_t len = sp.mono_len(m);
        R29 prod;
        if (len == 0) {
          prod = sp.c29[m];
        } else {
          for (uint32_t q = 0; q < len; q++) {
            const uint32_t s = sp.fac(f + q);
            const R29 lo = L.F[(s * PB + pl) * 2], hi = L.F[(s * PB + pl) * 2 + 1];
            R29 v;
            if constexpr (NP <= 4) {
              // lo + t (hi - lo + 4p): lazy, < 20p, then one carry pass
              const R29 d = norm29(sub29(hi, lo));
              R29 a = lo;
              if (t & 1u) a = add29(a, d);
              if (t & 2u) a = add29(a, add29(d, d));
              v = norm29(a);
            } else {
              v = add29(lo, mul29(sub29(hi, lo), sp.t29[t]));  // < 4p, lazy
              v = norm29(v);
            }
            prod = q == 0 ? v : mul29(prod, v);
          }
          if (!sp.skip(m) || len == 1) prod = mul29(prod, sp.c29[m]);
        }
        f += len;
        sum = red6p(add29(sum, prod));
      }
      acc = red6p(add29(acc, sum));
    }
    __syncthreads();
  }
}

// lazy value < 128p (limbs < 2^32) -> normalized, < 2p
QG_DEV R29 red128p(const R29& a) {
  R29 x = normfull29<FrP>(a);
  x = condsub29<FrP>(x, l9_mul_small(F29P<FrP>::P, 64));
  x = condsub29<FrP>(x, l9_mul_small(F29P<FrP>::P, 32));
  x = condsub29<FrP>(x, F29P<FrP>::KP20.k[16]);
  x = condsub29<FrP>(x, F29P<FrP>::P8);
  x = condsub29<FrP>(x, F29P<FrP>::P4);
  return condsub29<FrP>(x, F29P<FrP>::P2);
}

// Block sums of NP per-thread values acc[t] (each < 2p, normalized) -> res[t]
// (LDS, canonical words), visible to all threads on return.  All points move
// together (independent chains); additions are lazy, one parallel carry pass
// per shuffle step, one reduction per point at the wave and block levels.
// red: (blockDim / 64) * NP LDS scratch.
template <int NP>
QG_DEV void block_sums29(R29 (&acc)[NP], uint32_t np, R29* red, R29* res) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // one point at a time (register pressure of the sweep kernel stays low)
#pragma unroll
  for (int t = 0; t < NP; t++) {
    R29 a = acc[t];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) a = norm29(add29(a, shfl_xor29(a, m)));  // < 128p
    if (lane == 0 && (uint32_t)t < np) red[wid * NP + t] = red128p(a);
  }
  __syncthreads();
  if (threadIdx.x < np) {
    R29 a = red[threadIdx.x];
    for (uint32_t w = 1; w < nw; w++) a = add29(a, red[w * NP + threadIdx.x]);  // nw <= 8: < 16p
    res[threadIdx.x] = red16p29<FrP>(a);
  }
  __syncthreads();
}

// Sum of acc (< 2p, normalized) over the threads of each point t (t = tid %
// NP) -> res[t] (LDS, < 2p normalized), visible to all threads on return.
// Lazy: the shuffle steps and the cross-wave sum only add (with parallel
// carry passes); one reduction per point at the end.  red: (blockDim / 64) *
// NP LDS scratch.
template <int NP>
QG_DEV void block_reduce_pts(R29 acc, uint32_t np, R29* red, R29* res) {
#pragma unroll
  for (int m = 32; m >= NP; m >>= 1) acc = norm29(add29(acc, shfl_xor29(acc, m)));  // < 128p / NP
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane < NP) red[wid * NP + lane] = acc;
  __syncthreads();
  if (threadIdx.x < np) {
    // NP >= 4: a wave's value is < 32p; up to 4 of them (< 128p) between reductions
    R29 a = red[threadIdx.x];
    for (uint32_t w = 1; w < nw; w++) {
      if ((w & 3) == 0) a = red128p(a);
      a = norm29(add29(a, red[w * NP + threadIdx.x]));
    }
    res[threadIdx.x] = red128p(a);
  }
  __syncthreads();
}

// Sum of nrows rows of NP canonical values (row b at rows[b * NP]) -> res[t]
// (whole block; thread = (row group, point), lazy sums)
// All of a thread's rows (8 at 512 blocks) are in flight before any is added.
// Measured (micro/sc_trace.py "rows-summed"): 5.7 us for 512 rows either way --
// the time is not the load chain.
template <int NP>
QG_DEV void sum_rows29(const Fr* rows, uint32_t nrows, uint32_t np, R29* red, R29* res) {
  constexpr int BATCH = 8;  // one round trip for 512 rows at NP = 4
  const uint32_t t = threadIdx.x % NP, G = blockDim.x / NP;
  R29 a = R29::zero();
  if (t < np)
    for (uint32_t b0 = threadIdx.x / NP; b0 < nrows; b0 += BATCH * G) {
      Fr v[BATCH];
#pragma unroll
      for (int k = 0; k < BATCH; k++) {
        const uint32_t b = b0 + k * G;
        v[k] = b < nrows ? ld_sc1(rows + (size_t)b * NP + t) : Fr::zero();
      }
      // limbs: at most 7 normalized terms (< 2^29 each) between reductions
#pragma unroll
      for (int k = 0; k < 6; k++) a = add29(a, to29(v[k]));  // canonical: < p
      a = red16p29<FrP>(a);
#pragma unroll
      for (int k = 6; k < BATCH; k++) a = add29(a, to29(v[k]));
      a = red16p29<FrP>(a);
    }
  block_reduce_pts<NP>(a, np, red, res);
}

// Round bookkeeping.  The transcript state, the deferred absorb, the current
// challenge in 29-bit form and the last-block election counter live in one
// small device struct.
struct ScState {
  uint32_t state[8];  // absorbed transcript state
  uint32_t pend[20];  // state' || 48 challenge bytes of the last round, not yet absorbed
  uint32_t ticket;    // blocks of the current round that have published partials
  uint32_t err;       // persistent-kernel barrier timeout flag
  uint32_t r29[9];    // last challenge * 2^261 mod p (< 2p), the fold multiplier
  uint32_t pad[1];
  uint32_t claim[8];  // this round's claim h_{j-1}(r_{j-1}) at scale S (big rounds, j >= 1)
};

struct RoundOut {
  ScState* st;
  Fr* chal;          // nvars challenges (Montgomery, R = 2^256)
  Fr* coeffs;        // nvars x width (Montgomery)
  uint32_t* lens;    // nvars
  uint32_t width;    // row width (>= np)
};

struct FinSmem {
  uint32_t msg[144];  // state || u64 len || coefficients (canonical LE) || zero pad
  uint32_t chin[16];  // state' || "challenge" || zero pad
  uint32_t xof[16];   // B3-XOF(state' || "challenge")[0..64)
  uint32_t ab[32];    // state' || challenge bytes || zero pad (absorb)
  R29 r;              // the round challenge * 2^261 (fold multiplier)
  Fr r256;            // the round challenge (Montgomery, R = 2^256)
};

// Round message, transcript and challenge from the np round sums ev[] (LDS,
// canonical words at scale S).  Whole block calls (barriers); wave 0 works.
// Interpolation is lane-parallel over (coefficient t, node u): each lane
// multiplies by the inverse-Vandermonde entry scaled to give the Montgomery
// coefficient (proof output) and the canonical one (transcript bytes), then a
// shuffle sum over u.  Trim by ballot; BLAKE3 on one DPP quad; r from four
// lanes (r * 2^261 for the fold and r * 2^256 for the output, each lo + hi).
// Absorbing the 48 challenge bytes is deferred when pend_out != nullptr.
template <int NP>
// canon_out: the writer stores the CANONICAL coefficients (the transcript's) in
// ro.coeffs right away and skips the Montgomery pass after the challenge (the
// persistent tail: the host converts those rows, keeping ~1 us off every round)
QG_DEV void finish_core(const SopLds<NP>& sp, uint32_t np, const R29* ev, const RoundOut& ro,
                        uint32_t j, FinSmem& fs, const uint32_t* state_in, uint32_t* pend_out,
                        uint32_t* state_out, uint32_t tr = 4096, bool writer = true,
                        bool canon_out = false) {
  constexpr uint32_t U = NP <= 8 ? NP : 4;  // lanes per coefficient
  const uint32_t tid = threadIdx.x;
  const bool w0 = tid < 64;
  const uint32_t ct = tid / U, cu = tid % U;
  // canonical coefficients (transcript bytes) first; the Montgomery ones (proof
  // output) after the challenge.  Lazy sums: <= 4 terms < 2p per lane, U <= 8
  // lanes: < 64p before the one reduction.
  R29 cc = R29::zero();
  if (w0 && ct < np) {
    for (uint32_t u = cu; u < np; u += U) cc = add29(cc, mul29(sp.vc[ct * NP + u], ev[u]));
  }
  cc = norm29(cc);
#pragma unroll
  for (uint32_t m = 1; m < U; m <<= 1) cc = norm29(add29(cc, shfl_xor29(cc, m)));
  // U <= 8 products < 2p each: < 16p
  const Fr ccw = from29(canon29(red16p29<FrP>(cc)));
  const bool lead = w0 && cu == 0 && ct < np;
  if (writer && canon_out && lead) ro.coeffs[(size_t)j * ro.width + ct] = ccw;
  if (writer) {
    for (uint32_t i = np + tid; i < ro.width; i += blockDim.x)
      ro.coeffs[(size_t)j * ro.width + i] = Fr::zero();
  }
  const uint64_t nz = __ballot(lead && !ccw.is_zero());
  // highest nonzero coefficient: lane index / U + 1 (wave 0's ballot)
  const uint32_t len = nz ? (63u - (uint32_t)__clzll(nz)) / U + 1u : 0u;
  if (tid < 8) fs.msg[tid] = state_in[tid];
  if (lead) {
#pragma unroll
    for (int i = 0; i < 8; i++) fs.msg[10 + 8 * ct + i] = ccw.v[i];
  }
  for (uint32_t i = 10 + 8 * np + tid; i < 144; i += blockDim.x) fs.msg[i] = 0;
  if (tid == 0) {
    fs.msg[8] = len;
    fs.msg[9] = 0;
    fs.chin[8] = 0x6c616863u;  // "chal"
    fs.chin[9] = 0x676e656cu;  // "leng"
    fs.chin[10] = 0x00000065u; // "e"
  }
  if (tid >= 11 && tid < 16) fs.chin[tid] = 0;
  SC_TR(tr + 3);
  __syncthreads();
  // state' = B3(state || len || coefficients)
  if (w0) b3_hash_quad(fs.msg, 40 + 32 * len, fs.chin, 8);
  __syncthreads();
  SC_TR(tr + 4);
  // challenge bytes = B3-XOF(state' || "challenge")[0..48)
  if (w0) b3_hash_quad(fs.chin, 41, fs.xof, 16);
  __syncthreads();
  SC_TR(tr + 5);
  if (w0) {
    // r = lo + hi * 2^256 mod p (lo: bytes 0..31, hi: bytes 32..47)
    // lanes 0/1: lo * 2^522, hi * 2^778 -> r * 2^261; lanes 2/3: ... -> r * 2^256
    Fr x;
#pragma unroll
    for (int i = 0; i < 8; i++) x.v[i] = (tid & 1) ? (i < 4 ? fs.xof[8 + i] : 0u) : fs.xof[i];
    const R29 p = mul29(to29(x), sp.cr[tid & 3]);
    const R29 q = red6p(add29(p, shfl_xor29(p, 1)));
    if (tid == 0) fs.r = q;
    if (tid == 2) {
      const Fr rr = from29(canon29(q));
      fs.r256 = rr;
      if (writer) {
        ro.chal[j] = rr;
        ro.lens[j] = len;
      }
    }
  }
  if (pend_out) {
    if (tid < 20) pend_out[tid] = tid < 8 ? fs.chin[tid] : fs.xof[tid - 8];
  } else {
    if (tid < 32) fs.ab[tid] = tid < 8 ? fs.chin[tid] : (tid < 20 ? fs.xof[tid - 8] : 0u);
  }
  __syncthreads();
  SC_TR(tr + 6);
  if (!pend_out && w0) b3_hash_quad(fs.ab, 80, state_out, 8);
  if (writer && !canon_out) {
    // Montgomery coefficients for the proof output (off the challenge path)
    R29 cm = R29::zero();
    if (w0 && ct < np) {
      for (uint32_t u = cu; u < np; u += U) cm = add29(cm, mul29(sp.vm[ct * NP + u], ev[u]));
    }
    cm = norm29(cm);
#pragma unroll
    for (uint32_t m = 1; m < U; m <<= 1) cm = norm29(add29(cm, shfl_xor29(cm, m)));
    if (lead) ro.coeffs[(size_t)j * ro.width + ct] = from29(canon29(red128p(cm)));
  }
}

// round kernel: fused fold(r_{j-1}) + evaluate at t = 0..np-1, per-block
// partial sums; the last block to publish (ticket election) sums the partials
// and, with loc == nullptr, runs the round's transcript step itself; with
// loc != nullptr (sharded) it writes this rank's local sums for the allgather.
template <int K, int NP>
__global__ void __launch_bounds__(SC_BLOCK)
    k_sc_round(TablePtrs tp, const SopDev* __restrict__ spg, SopHdr h, size_t npairs, int fold,
               RoundOut ro, uint32_t j, int pending, Fr* __restrict__ partial, Fr* __restrict__ loc) {
  __shared__ SopLds<NP> sp;
  __shared__ RoundLds<K, NP, SC_BLOCK> L;
  __shared__ R29 red[(SC_BLOCK / 64) * NP];
  __shared__ R29 res[NP];
  __shared__ FinSmem fs;
  __shared__ uint32_t last;
  const uint32_t tid = threadIdx.x;
  const uint32_t tr = 1024 + 16 * j;
  if (blockIdx.x == 0) SC_TR(tr + 0);
  sop_load<NP>(sp, spg, h, loc == nullptr);
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (tid == (uint32_t)i) {
      L.src[i] = tp.src[i];
      L.dst[i] = tp.dst[i];
    }
  }
  R29 r = R29::zero();
  if (fold) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = ro.st->r29[i];
  }
  if (pending && blockIdx.x == 0 && tid >= 64 && tid < 128) {
    // deferred absorb of round j-1's challenge bytes (wave 1 of block 0),
    // handed to the last block write-through (see k_sc_big)
    if (tid - 64 < 32) fs.ab[tid - 64] = tid - 64 < 20 ? ro.st->pend[tid - 64] : 0u;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    b3_hash_quad(fs.ab, 80, fs.chin, 8);
    __builtin_amdgcn_wave_barrier();
    if (tid - 64 < 8) st_sc1_u32(&ro.st->state[tid - 64], fs.chin[tid - 64]);
  }
  __syncthreads();
  constexpr uint32_t PB = SC_BLOCK / NP;
  R29 acc = R29::zero();
  round_sweep<K, NP, SC_BLOCK>(L, sp, h, npairs, fold != 0, r, (size_t)blockIdx.x * PB,
                               (size_t)gridDim.x * PB, acc);
  if (blockIdx.x == 0) SC_TR(tr + 1);
  block_reduce_pts<NP>(acc, h.np, red, res);
  if (tid < h.np) st_sc1(partial + (size_t)blockIdx.x * NP + tid, from29(canon29(res[tid])));
  drain_stores();
  __syncthreads();
  if (tid == 0) {
    const uint32_t old = __hip_atomic_fetch_add((gu32*)&ro.st->ticket, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    last = old + 1 == gridDim.x;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  __syncthreads();
  if (!last) return;
  SC_TR(tr + 2);
  __shared__ uint32_t st_in[8];
  if (tid < 8) st_in[tid] = ld_sc1_u32(&ro.st->state[tid]);
  acc = R29::zero();
  {
    const uint32_t t = tid % NP;
    if (t < h.np)
      for (uint32_t b = tid / NP; b < gridDim.x; b += SC_BLOCK / NP)
        acc = red6p(add29(acc, to29(ld_sc1(partial + (size_t)b * NP + t))));
  }
  block_reduce_pts<NP>(acc, h.np, red, res);
  if (tid == 0) ro.st->ticket = 0;
  if (loc) {
    if (tid < NP) loc[tid] = tid < h.np ? from29(canon29(res[tid])) : Fr::zero();
    return;
  }
  finish_core<NP>(sp, h.np, res, ro, j, fs, st_in, ro.st->pend, nullptr, tr, true, true);
  if (tid < 9) ro.st->r29[tid] = fs.r.l[tid];
  SC_TR(tr + 7);
}

// ---------------------------------------------------------------------------
// Throughput form of a large round for product expressions (SOP_PURE, e.g.
// the h = g1 g2 g3 of config 3): one thread per pair (grid-stride), no LDS
// staging and no per-step barriers.  Slot by slot the thread folds its 4
// entries by r_{j-1} (2 throughput multiplies; the folded pair is written back
// < 2p) and multiplies lo + t (hi - lo) into the running product of every
// point t = 0..np-1; the points accumulate lazily.  Other expressions use the
// LDS-staged k_sc_round.
// ---------------------------------------------------------------------------

// Barrier over the G blocks of the slice tail with its arrival counter split
// in 8 shards (block b adds to shard b % 8, its XCD under round-robin
// dispatch; each shard on its own 128-B line): a few dozen arrivals per line
// instead of G on one.  The counters run cumulatively through the launch
// (`target` = all arrivals so far), zeroed by the host per call.  Every wave
// drains its stores and atomics first; the poll reads every shard (sc1).
QG_DEV void grid_barrier8(uint32_t* bar8, uint32_t target, uint32_t* err) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add((gu32*)(bar8 + 32 * (blockIdx.x & 7)), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
    for (;;) {
      uint32_t v[8], sum = 0;
#pragma unroll
      for (int x = 0; x < 8; x++) v[x] = ld_sc1_u32(bar8 + 32 * x);
#pragma unroll
      for (int x = 0; x < 8; x++) sum += v[x];
      if (sum >= target) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 26)) {
        st_sc1_u32(err, 1u);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps loads below
  }
  __syncthreads();
}

// u64 sums of normalized 29-bit limbs (each sum < 2^40) -> the value mod p,
// < 2p normalized.  T = L + c 2^261 with L < 2^261 and c < 32 when T is a sum
// of fewer than 2720 values < 2p; 2^261 = ONE (mod p), so T = L + c ONE < 202p.
QG_DEV R29 limbsum29(const uint64_t* a) {
  R29 x;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint64_t v = a[i] + c;
    x.l[i] = (uint32_t)v & M29;
    c = v >> 29;
  }
  x = normfull29<FrP>(add29(x, R29::from_l9(l9_mul_small(F29P<FrP>::ONE, (uint32_t)c))));
  x = condsub29<FrP>(x, l9_mul_small(F29P<FrP>::P, 128));
  return red128p(x);
}

// ---------------------------------------------------------------------------
// Large rounds, thread per pair (k_sc_big).
//  * Sweep: one thread per pair, grid-stride.  Slot by slot the thread folds
//    its 4 entries by r_{j-1} (throughput multiplies; the folded pair is
//    written back < 2p) and evaluates at t = 0..np-1: product expressions
//    (SOP_PURE) multiply lo + t (hi - lo) into a running product per point,
//    the next slot's entries in flight during the current slot's arithmetic;
//    other expressions (K <= 4) keep every slot's lo / hi and run the
//    compiled monomials with uniform-index selects.  The points accumulate
//    lazily (three additions per reduction).
//  * Round end: per-block partial rows; the last block to publish (ticket)
//    sums them and runs the transcript step.
// ---------------------------------------------------------------------------
// lo + t (hi - lo + 4p) for point t (d = norm29(hi - lo + 4p) < 6p)
// the same value left lazy (limbs < 2^31 + 32, value < 20p) for NP <= 4: a
// multiplier operand next to a normalized one (< 2p) keeps every column below
// 2^64 and the product below 1.3p, so only the first factor needs the carry pass
template <int NP>
QG_DEV R29 at_point_lazy(const R29& lo, const R29& d, int t, const SopLds<NP>& sp) {
  if constexpr (NP <= 4) {
    R29 v = lo;
    if (t & 1) v = add29(v, d);
    if (t & 2) v = add29(v, add29(d, d));
    return v;
  } else {
    return norm29(add29(lo, mul29t(d, sp.t29[t])));
  }
}

template <int NP>
QG_DEV R29 at_point(const R29& lo, const R29& d, int t, const SopLds<NP>& sp) {
  if constexpr (NP <= 4) {
    R29 v = lo;  // lazy, < 20p, then one carry pass
    if (t & 1) v = add29(v, d);
    if (t & 2) v = add29(v, add29(d, d));
    return norm29(v);
  } else {
    return norm29(add29(lo, mul29t(d, sp.t29[t])));  // < 4p
  }
}

// fold x0..x3 -> (lo, hi) < 2p and store them (round j >= 1), or take x0, x1.
// Bounds: x < 2p, x1 - x0 + 4p < 6p, r < 2p: the product is < 12p^2/2^261 + p
// < 1.1p, so x0 + it < 3.1p and one conditional subtraction of 2p suffices.
QG_DEV void fold_pair(const Fr (&w)[4], bool fold, const R29& r, Fr* dst, R29& lo, R29& hi) {
  if (fold) {
    const R29 x0 = to29(w[0]), x1 = to29(w[1]), x2 = to29(w[2]), x3 = to29(w[3]);
#ifndef QG_SC_NO_ILP
    // the two products interleaved (field29.h mul29tn): no dependent-mad nops
    R29 a[2] = {sub29(x1, x0), sub29(x3, x2)}, b[2] = {r, r};
    mul29tn<FrP, 2>(a, b, a);
    lo = red2p29<FrP>(add29(x0, a[0]));
    hi = red2p29<FrP>(add29(x2, a[1]));
#else
    lo = red2p29<FrP>(add29(x0, mul29t(sub29(x1, x0), r)));
    hi = red2p29<FrP>(add29(x2, mul29t(sub29(x3, x2), r)));
#endif
    dst[0] = from29(lo);
    dst[1] = from29(hi);
  } else {
    lo = to29(w[0]);
    hi = to29(w[1]);
  }
}

QG_DEV void load_pair(const Fr* src, bool fold, Fr (&w)[4]) {
  w[0] = src[0];
  w[1] = src[1];
  if (fold) {
    w[2] = src[2];
    w[3] = src[3];
  }
}

template <int K>
QG_DEV R29 pick29(const R29 (&v)[K], uint32_t i) {
  // select chain on a uniform index (v_cndmask): a switch of loads would be
  // merged into one dynamically indexed load and demote v[] to scratch
  i = __builtin_amdgcn_readfirstlane(i);
  R29 r = v[0];
#pragma unroll
  for (int k = 1; k < K; k++)
    if (i == (uint32_t)k) r = v[k];
  return r;
}

// source / destination tables of round j of k_sc_big: round 0 reads the
// input tables; round j >= 1 folds into X (j odd, N/2 per slot) or Y (j even,
// N/4 per slot) and reads round j - 1's output
struct AllBufs {
  TablePtrs in;  // src[] = input tables
  Fr* X;
  Fr* Y;
  size_t capX, capY;
  QG_DEV const Fr* src(uint32_t j, uint32_t s) const {
    if (j <= 1) return in.src[s];
    return (j & 1) ? Y + capY * s : X + capX * s;
  }
  QG_DEV Fr* dst(uint32_t j, uint32_t s) const { return (j & 1) ? X + capX * s : Y + capY * s; }
};

template <int K, int NP, bool PURE>
QG_DEV void sweep_pairs(const AllBufs& tb, uint32_t j, bool fold, const R29& r, size_t npairs,
                        size_t p0, size_t stride, const SopLds<NP>& sp, const SopHdr& h,
                        bool skip0, R29 (&acc)[NP]) {
  const uint32_t nslots = h.nslots, np = h.np;
  uint32_t cnt = 0;
  if constexpr (PURE) {
    // one pair: fold the slots, multiply the points, accumulate lazily
    // (prefetching the next slot's and the next pair's entries during the
    // current slot was measured slower: +14 us over the big rounds at 2^20,
    // profiles/r04_sumcheck_prefetch_ab.txt)
    auto body = [&](size_t p) {
      R29 prod[NP];
      Fr w[4];
      for (uint32_t s = 0; s < nslots; s++) {
        load_pair(tb.src(j, s) + (fold ? 4 : 2) * p, fold, w);
        R29 lo, hi;
        fold_pair(w, fold, r, tb.dst(j, s) + 2 * p, lo, hi);
        const R29 d = norm29(sub29(hi, lo));
#ifndef QG_SC_NO_ILP
        if constexpr (NP == 4) {
          // the point products as interleaved chains (field29.h mul29tn): 4
          // (round 0) or 3 (skip0: t = 1..3) independent multiplies in flight
          if (s == 0) {
#pragma unroll
            for (int t = 0; t < NP; t++) prod[t] = at_point<NP>(lo, d, t, sp);
          } else if (skip0) {
            R29 a[3] = {prod[1], prod[2], prod[3]};
            R29 b[3] = {at_point_lazy<NP>(lo, d, 1, sp), at_point_lazy<NP>(lo, d, 2, sp),
                        at_point_lazy<NP>(lo, d, 3, sp)};
            mul29tn<FrP, 3>(a, b, a);
            prod[1] = a[0];
            prod[2] = a[1];
            prod[3] = a[2];
          } else {
            R29 b[4];
#pragma unroll
            for (int t = 0; t < NP; t++) b[t] = at_point_lazy<NP>(lo, d, t, sp);
            mul29tn<FrP, 4>(prod, b, prod);
          }
        } else
#endif
        {
#pragma unroll
          for (int t = 0; t < NP; t++) {
            if (t == 0 && skip0) continue;  // h(0) = claim - h(1), by the finisher
            if (s == 0)
              prod[t] = at_point<NP>(lo, d, t, sp);
            else
              prod[t] = mul29t(prod[t], at_point_lazy<NP>(lo, d, t, sp));
          }
        }
      }
      // products of >= 2 factors are < 4p: three lazy additions stay below 16p
#pragma unroll
      for (int t = 0; t < NP; t++)
        if ((uint32_t)t < np && !(t == 0 && skip0)) acc[t] = add29(acc[t], prod[t]);
      if (++cnt == 3) {
#pragma unroll
        for (int t = 0; t < NP; t++) acc[t] = red16p29<FrP>(acc[t]);
        cnt = 0;
      }
    };
    for (size_t p = p0; p < npairs; p += stride) body(p);

  } else {
  for (size_t p = p0; p < npairs; p += stride) {
    R29 prod[NP];
    {
      static_assert(PURE || K <= 4, "generic sweep keeps <= 4 slots in registers");
      R29 lo[K], hi[K], dd[K];
#pragma unroll
      for (int s = 0; s < K; s++) {
        lo[s] = hi[s] = dd[s] = R29::zero();
        if ((uint32_t)s < nslots) {
          Fr w[4];
          load_pair(tb.src(j, s) + (fold ? 4 : 2) * p, fold, w);
          fold_pair(w, fold, r, tb.dst(j, s) + 2 * p, lo[s], hi[s]);
          dd[s] = norm29(sub29(hi[s], lo[s]));
        }
      }
      uint32_t f = 0;
      for (uint32_t m = 0; m < h.nmono; m++) {
        const uint32_t len = sp.mono_len(m);
        if (len == 0) {
#pragma unroll
          for (int t = 0; t < NP; t++) prod[t] = sp.c29[m];
        } else {
          for (uint32_t q = 0; q < len; q++) {
            const uint32_t s = sp.fac(f + q);
            const R29 a = pick29<K>(lo, s), d = pick29<K>(dd, s);
#pragma unroll
            for (int t = 0; t < NP; t++) {
              if (t == 0 && skip0) continue;
              const R29 v = at_point<NP>(a, d, t, sp);
              prod[t] = q == 0 ? v : mul29t(prod[t], v);
            }
          }
          if (!sp.skip(m) || len == 1) {
#pragma unroll
            for (int t = 0; t < NP; t++)
              if (!(t == 0 && skip0)) prod[t] = mul29t(prod[t], sp.c29[m]);
          }
        }
        f += len;
        // every monomial value is < 4p (a single factor is scaled by its
        // multiplier): three lazy additions stay below 16p
#pragma unroll
        for (int t = 0; t < NP; t++)
          if ((uint32_t)t < np && !(t == 0 && skip0)) acc[t] = add29(acc[t], prod[t]);
        if (++cnt == 3) {
#pragma unroll
          for (int t = 0; t < NP; t++) acc[t] = red16p29<FrP>(acc[t]);
          cnt = 0;
        }
      }
    }
  }
  }
#pragma unroll
  for (int t = 0; t < NP; t++) acc[t] = red16p29<FrP>(acc[t]);
}

// One large round (tables > 2^PERS_LOG) in one launch: thread-per-pair sweep
// (sweep_pairs), per-block partial rows, and the last block to publish
// (ticket election) sums the rows and runs the transcript step (or, sharded,
// writes this rank's local sums).
template <int K, int NP, bool PURE, int WPE = 1>
__global__ void __launch_bounds__(SC_BLOCK) __attribute__((amdgpu_waves_per_eu(WPE)))
    k_sc_big(AllBufs tb, uint32_t j, const SopDev* __restrict__ spg, SopHdr h, size_t npairs,
             RoundOut ro, int pending, Fr* __restrict__ loc, int skip0, uint64_t* __restrict__ acc_j,
             uint64_t* __restrict__ acc_next, uint32_t* __restrict__ bar8) {
  __shared__ SopLds<NP> sp;
  __shared__ R29 red[(SC_BLOCK / 64) * NP];
  __shared__ R29 res[NP];
  __shared__ FinSmem fs;
  __shared__ uint32_t last;
  __shared__ uint64_t lsum[NP * 9];
  const uint32_t tid = threadIdx.x;
  const uint32_t tr = 1024 + 16 * j;
  const bool fold = j > 0;
  if (blockIdx.x == 0) SC_TR(tr + 0);
  SC_TB(j, 0);
  sop_load<NP>(sp, spg, h, loc == nullptr);
  R29 r = R29::zero();
  if (fold) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = ro.st->r29[i];
  }
  if (pending && blockIdx.x == 0 && tid >= 64 && tid < 128) {
    // deferred absorb of round j-1's challenge bytes (wave 1 of block 0); the
    // new state is handed to the last block write-through (sc1) and drained
    // before this block's ticket
    if (tid - 64 < 32) fs.ab[tid - 64] = tid - 64 < 20 ? ro.st->pend[tid - 64] : 0u;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    b3_hash_quad(fs.ab, 80, fs.chin, 8);
    __builtin_amdgcn_wave_barrier();
    if (tid - 64 < 8) st_sc1_u32(&ro.st->state[tid - 64], fs.chin[tid - 64]);
  }
  if (skip0 && blockIdx.x == 0 && tid == 128) {
    // this round's claim h_{j-1}(r_{j-1}) at scale S, for the finisher's
    // h(0) = claim - h(1): Horner over round j-1's canonical coefficients
    // (wave 2 of block 0, beside the sweep; handed over write-through)
    const Fr* c = ro.coeffs + (size_t)(j - 1) * ro.width;
    R29 a = to29(c[h.np - 1]);
    for (int t = (int)h.np - 2; t >= 0; t--) a = red6p(add29(mul29(a, r), to29(c[t])));
    R29 cs;
#pragma unroll
    for (int i = 0; i < 9; i++) cs.l[i] = spg->cs29.v[i];
    st_sc1(reinterpret_cast<Fr*>(ro.st->claim), from29(canon29(red6p(mul29(a, cs)))));
  }
  __syncthreads();
  const uint32_t np = h.np;
  R29 acc[NP];
#pragma unroll
  for (int t = 0; t < NP; t++) acc[t] = R29::zero();
  sweep_pairs<K, NP, PURE>(tb, j, fold, r, npairs, (size_t)blockIdx.x * SC_BLOCK + tid,
                               (size_t)gridDim.x * SC_BLOCK, sp, h, skip0 != 0, acc);
  if (blockIdx.x == 0) SC_TR(tr + 1);
  SC_TB(j, 1);
  SC_TW(j);
  block_sums29<NP>(acc, np, red, res);
  // publish: the limbs of the block sums added into this round's accumulator
  // shard (agent-scope u64 atomics, executed at the memory side), every wave
  // drains, then a two-level ticket: the block completing its shard (blocks b
  // with b % 8 = x, one 128-B counter line per shard) adds to the round's
  // ticket, and the one completing that is the last block
  if (tid < np * 9)
    __hip_atomic_fetch_add((gu64*)(acc_j + (blockIdx.x & 7) * (16 * 9) + tid),
                           (uint64_t)res[tid / 9].l[tid % 9], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  drain_stores();
  __syncthreads();
  if (tid == 0) {
    const uint32_t x = blockIdx.x & 7, nx = (gridDim.x + 7 - x) / 8;
    bool done = false;
    const uint32_t o1 = __hip_atomic_fetch_add((gu32*)(bar8 + 32 * x), 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT);
    if (o1 + 1 == nx) {
      const uint32_t o2 = __hip_atomic_fetch_add((gu32*)&ro.st->ticket, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
      done = o2 + 1 == (gridDim.x < 8 ? gridDim.x : 8u);
    }
    last = done;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: loads stay below
  }
  __syncthreads();
  if (!last) return;
  SC_TR(tr + 2);
  __shared__ uint32_t st_in[8];
  if (tid < 8) st_in[tid] = ld_sc1_u32(&ro.st->state[tid]);
  if (tid < np * 9) {
    uint64_t v[8], a = 0;
#pragma unroll
    for (int x = 0; x < 8; x++)
      v[x] = __hip_atomic_fetch_add((gu64*)(acc_j + x * (16 * 9) + tid), (uint64_t)0,
                                    __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int x = 0; x < 8; x++) a += v[x];
    lsum[tid] = a;
  }
  __syncthreads();
  if (tid < np) res[tid] = limbsum29(lsum + 9 * tid);
  // counters back to zero and the next round's accumulator cleared (the next
  // kernel on the stream sees both)
  if (tid < 8) st_sc1_u32(bar8 + 32 * tid, 0u);
  for (uint32_t i = tid; i < 8 * 16 * 9; i += SC_BLOCK)
    __hip_atomic_store((gu64*)(acc_next + i), (uint64_t)0, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  SC_TR(tr + 8);
  if (tid == 0) ro.st->ticket = 0;
  if (loc) {  // sharded: k_sc_finish applies the claim to the global sums
    if (tid < NP) loc[tid] = tid < np ? from29(canon29(res[tid])) : Fr::zero();
    return;
  }
  if (skip0 && tid == 0)
    res[0] = red6p(sub29(to29(ld_sc1(reinterpret_cast<const Fr*>(ro.st->claim))), res[1]));
  __syncthreads();
  finish_core<NP>(sp, np, res, ro, j, fs, st_in, ro.st->pend, nullptr, tr, true, true);
  if (tid < 9) ro.st->r29[tid] = fs.r.l[tid];
  SC_TR(tr + 7);
}

// sharded: the transcript step over the allgathered [rank][NP] local sums
template <int NP>
__global__ void __launch_bounds__(SC_BLOCK)
    k_sc_finish(const SopDev* __restrict__ spg, SopHdr h, const Fr* __restrict__ rows,
                uint32_t nrows, RoundOut ro, uint32_t j, int skip0) {
  __shared__ SopLds<NP> sp;
  __shared__ R29 red[(SC_BLOCK / 64) * NP];
  __shared__ R29 res[NP];
  __shared__ FinSmem fs;
  __shared__ uint32_t st[8];
  const uint32_t tid = threadIdx.x;
  sop_load<NP>(sp, spg, h, true);
  if (tid < 8) st[tid] = ro.st->state[tid];
  R29 acc = R29::zero();
  {
    const uint32_t t = tid % NP;
    if (t < h.np)
      for (uint32_t b = tid / NP; b < nrows; b += SC_BLOCK / NP)
        acc = red6p(add29(acc, to29(rows[(size_t)b * NP + t])));
  }
  __syncthreads();
  block_reduce_pts<NP>(acc, h.np, red, res);
  if (skip0 && tid == 0)  // h(0) = claim - h(1) on the global sums
    res[0] = red6p(sub29(to29(*reinterpret_cast<const Fr*>(ro.st->claim)), res[1]));
  __syncthreads();
  finish_core<NP>(sp, h.np, res, ro, j, fs, st, nullptr, ro.st->state, 4096, true, true);
  if (tid < 9) ro.st->r29[tid] = fs.r.l[tid];
}

// Grid barrier among the first n blocks (monotonic per-round counter): every
// wave drains its sc1 stores, one lane adds to the counter and polls it with
// sc1 loads, the others wait at the workgroup barrier.  Everything handed
// across it is stored and loaded sc1 (helpers above), so no fences.  The spin
// is bounded: on timeout the error flag is raised and the kernel runs on to
// its end (the host reports QG_ERR_DEVICE).
QG_DEV void grid_barrier(uint32_t* ctr, uint32_t n, uint32_t* err) {
  drain_stores();
  __syncthreads();
  if (threadIdx.x == 0) {
    gu32* c = (gu32*)ctr;
    __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < n) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 26)) {
        st_sc1_u32(err, 1u);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps loads below
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Persistent tail: rounds j0..nvars-1 in ONE launch of TAIL_BLOCK-thread workgroups,
// one per CU.  Round j keeps nb_j = ceil(pairs / PB) blocks (PB pairs per
// block step; the others retire), each sweeps its pairs (phase F: fold into
// the LDS staging array F and, while other blocks read them next round, into
// HBM with sc1 stores; phase E: thread (pair, point) evaluates h), publishes
// its per-point sums, meets the others at the grid barrier, then every block
// sums the partials and runs the identical transcript step — no second
// barrier, no broadcast.  Block 0 writes the proof outputs.
// Once a round fits one block step (nb == 1, pairs <= PB) its folded table IS
// the staging array, so from the next round on the tables never leave LDS:
// F ping-pongs between two arrays (the second half as large: the table halves
// every round), no HBM round trip, no barrier.  The deferred absorb of the
// previous challenge runs on the block's LAST wave, which has no pair work in
// the small rounds, beside the sweep.  Final fold + claim by block 0.
// PB is chosen at run time from the slot count (tail_pb, shared with the
// host's grid computation) so the two staging arrays fit TAIL_FBYTES.
static constexpr int TAIL_BLOCK = 256;
static constexpr uint32_t TAIL_FBYTES = 32 * 1024;  // LDS for the staging arrays
// np: the kernel's point stride NP (threads per pair), not the expression's np
QG_HD uint32_t tail_pb(uint32_t nslots, uint32_t np) {
  // F0: nslots x 2 PB entries, F1: nslots x PB entries, 36 B each
  const uint32_t per = nslots ? nslots * 108u : 108u;
  uint32_t pb = 1;
  while (pb * 2 * per <= TAIL_FBYTES && pb * 2 * np <= (uint32_t)TAIL_BLOCK) pb *= 2;
  return pb;
}

// Per-point sums when only the first `n` threads (n <= 64: wave 0) hold
// values: a shuffle tree of exactly log2(n / NP) steps inside wave 0, no LDS
// staging; else the block reduction.  res[t] (LDS, < 2p) on return.
template <int NP>
QG_DEV void tail_reduce(R29 acc, uint32_t n, uint32_t np, R29* red, R29* res) {
  uint32_t n2 = NP;
  while (n2 < n) n2 <<= 1;  // lanes past n hold zeros
  if (n2 > 64) {
    block_reduce_pts<NP>(acc, np, red, res);
    return;
  }
  if (threadIdx.x < 64) {
    for (uint32_t m = n2 / 2; m >= NP; m >>= 1) acc = norm29(add29(acc, shfl_xor29(acc, m)));
    if (threadIdx.x < np) res[threadIdx.x] = red128p(acc);
  }
  __syncthreads();
}

template <int NP>
QG_DEV void tail_eval(const R29* F, uint32_t ss, const SopLds<NP>& sp, const SopHdr& h,
                      uint32_t pl, uint32_t t, R29& acc) {
  R29 sum = R29::zero();
  uint32_t f = 0;
  for (uint32_t m = 0; m < h.nmono; m++) {
    const uint32_t len = sp.mono_len(m);
    R29 prod;
    if (len == 0) {
      prod = sp.c29[m];
    } else {
      for (uint32_t q = 0; q < len; q++) {
        const uint32_t s = sp.fac(f + q);
        const R29 lo = F[s * ss + 2 * pl], hi = F[s * ss + 2 * pl + 1];
        R29 v;
        if constexpr (NP <= 4) {
          const R29 d = norm29(sub29(hi, lo));
          R29 a = lo;
          if (t & 1u) a = add29(a, d);
          if (t & 2u) a = add29(a, add29(d, d));
          v = q == 0 ? norm29(a) : a;  // later factors stay lazy (see at_point_lazy)
        } else {
          v = norm29(add29(lo, mul29(sub29(hi, lo), sp.t29[t])));
        }
        prod = q == 0 ? v : mul29(prod, v);
      }
      if (!sp.skip(m) || len == 1) prod = mul29(prod, sp.c29[m]);
    }
    f += len;
    sum = red6p(add29(sum, prod));
  }
  acc = red6p(add29(acc, sum));
}

template <int K, int NP>
__global__ void __launch_bounds__(TAIL_BLOCK)
    k_sc_tail(TablePtrs tp0, TablePtrs bufA, TablePtrs bufB, const SopDev* __restrict__ spg,
              SopHdr h, uint32_t nvars, uint32_t j0, int fold0, int pending0, RoundOut ro,
              Fr* __restrict__ partial, uint32_t* __restrict__ bar, Fr* __restrict__ final_vals,
              Fr* __restrict__ evaluation) {
  __shared__ SopLds<NP> sp;
  __shared__ R29 Fbuf[TAIL_FBYTES / sizeof(R29)];
  __shared__ R29 red[(TAIL_BLOCK / 64) * NP];
  __shared__ R29 res[NP];
  __shared__ FinSmem fs;
  __shared__ uint32_t st[8];
  __shared__ uint32_t pend[32];
  const uint32_t tid = threadIdx.x, blk = blockIdx.x;
  const uint32_t nslots = h.nslots, np = h.np;
  const uint32_t PB = tail_pb(nslots, NP);  // (pair, point) threads: NP per pair
  const uint32_t t = tid % NP, pl = tid / NP;
  const bool writer = blk == 0;
  const bool last_wave = tid >= TAIL_BLOCK - 64;
  // F0 (slot stride 2 PB) and F1 (slot stride PB)
  R29* const F0 = Fbuf;
  R29* const F1 = Fbuf + (size_t)(nslots ? nslots : 1) * 2 * PB;
  sop_load<NP>(sp, spg, h, true);
  if (tid < 8) st[tid] = ro.st->state[tid];
  if (tid < 32) pend[tid] = (pending0 && tid < 20) ? ro.st->pend[tid] : 0u;
  R29 r = R29::zero();
  if (fold0) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = ro.st->r29[i];
  }
  __syncthreads();
  TablePtrs cur = tp0;
  int fold = fold0, pending = pending0;
  // where this round's source lives: HBM (cur.src) or LDS (prev, slot stride ss_prev)
  const R29* prev = nullptr;
  uint32_t ss_prev = 0;
  R29* wr = F0;
  uint32_t ss_wr = 2 * PB;
  for (uint32_t j = j0; j < nvars; j++) {
    const size_t npairs = (size_t)1 << (nvars - 1 - j);
    const uint32_t nb = (uint32_t)std::min<size_t>(gridDim.x, (npairs + PB - 1) / PB);
    if (blk >= nb) return;  // retired: every later round has fewer pairs
    const bool single = nb == 1 && npairs <= PB;
    if (writer) SC_TR(16 * j + 0);
    if (pending && last_wave) b3_hash_quad(pend, 80, st, 8);  // beside the sweep
    // ---- phase F: fold (or copy) this round's table into the staging array
    R29 acc = R29::zero();
    const size_t stride = (size_t)nb * PB;
    for (size_t base = (size_t)blk * PB; base < npairs; base += stride) {
      const uint32_t cnt = (uint32_t)std::min<size_t>(PB, npairs - base);
      const uint32_t per = 2 * cnt, nitems = nslots * per;
      for (uint32_t it = tid; it < nitems; it += TAIL_BLOCK) {
        const uint32_t s = it / per, e = it % per;
        const size_t idx = 2 * base + e;  // entry of this round's (folded) table
        R29 v;
        if (prev) {  // LDS-resident source: entries 2e, 2e+1 of the previous table
          const R29 x0 = prev[s * ss_prev + 2 * e], x1 = prev[s * ss_prev + 2 * e + 1];
          v = red2p29<FrP>(add29(x0, mul29(sub29(x1, x0), r)));
        } else if (fold) {
          const Fr* src = cur.src[s] + 2 * idx;
          const R29 x0 = to29(ld_sc1(src)), x1 = to29(ld_sc1(src + 1));
          v = red2p29<FrP>(add29(x0, mul29(sub29(x1, x0), r)));
          if (!single) st_sc1(cur.dst[s] + idx, from29(v));
        } else {
          v = to29(ld_sc1(cur.src[s] + idx));
        }
        wr[s * ss_wr + e] = v;
      }
      __syncthreads();
      // ---- phase E: thread (pair pl, point t)
      if (t < np && pl < cnt) tail_eval<NP>(wr, ss_wr, sp, h, pl, t, acc);
      if (base + stride < npairs) __syncthreads();  // the staging array is refilled
    }
    if (writer) SC_TR(16 * j + 1);
    {
      // threads holding values: NP per pair of this block's (last) step
      const size_t first = (size_t)blk * PB;
      const uint32_t cnt = npairs > first ? (uint32_t)std::min<size_t>(PB, npairs - first) : 0u;
      tail_reduce<NP>(acc, npairs > stride ? (uint32_t)TAIL_BLOCK : cnt * NP, np, red, res);
    }
    if (writer) SC_TR(16 * j + 7);
    if (nb > 1) {
      Fr* part = partial + (size_t)(j & 1) * gridDim.x * NP;
      if (tid < np) st_sc1(part + (size_t)blk * NP + tid, from29(canon29(res[tid])));
      grid_barrier(bar + j, nb, &ro.st->err);
      if (writer) SC_TR(16 * j + 8);
      acc = R29::zero();
      if (t < np)
        for (uint32_t b0 = pl; b0 < nb; b0 += 4 * (TAIL_BLOCK / NP)) {
          // four partials in flight at once, then acc (< 2p) + 4 values (< p) < 6p
          Fr v[4];
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const uint32_t b = b0 + k * (TAIL_BLOCK / NP);
            v[k] = b < nb ? ld_sc1(part + (size_t)b * NP + t) : Fr::zero();
          }
#pragma unroll
          for (int k = 0; k < 4; k++) acc = add29(acc, to29(v[k]));
          acc = red6p(acc);
        }
      // rows of nb blocks: thread (row pl, point t) holds one when nb * NP <= 64
      tail_reduce<NP>(acc, std::min<uint32_t>(nb, TAIL_BLOCK / NP) * NP, np, red, res);
    }
    if (writer) SC_TR(16 * j + 2);
    finish_core<NP>(sp, np, res, ro, j, fs, st, pend, nullptr, writer ? 16 * j : 4096, writer,
                    true);
    __syncthreads();
    r = fs.r;
    pending = 1;
    // next round's source: the staging array just written when this round was a
    // single block step, else the HBM tables this round folded into
    if (single) {
      prev = wr;
      ss_prev = ss_wr;
      const bool w0 = wr == F0;
      wr = w0 ? F1 : F0;
      ss_wr = w0 ? PB : 2 * PB;
    } else {
      TablePtrs nxt;
      const TablePtrs& w = ((j - j0) & 1) ? bufB : bufA;
      for (int i = 0; i < 8; i++) {
        nxt.src[i] = fold ? cur.dst[i] : cur.src[i];
        nxt.dst[i] = w.dst[i];
      }
      cur = nxt;
    }
    fold = 1;
  }
  // final fold with r_{n-1} on the 32-bit path: the last round (one pair) is
  // always a single block step, so its two folded entries per slot are in prev
  if (tid == 0) {
    const Fr rr = fs.r256;
    Fr val[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
      if ((uint32_t)i < nslots) {
        const Fr a = lt_p(from29(prev[i * ss_prev])), b = lt_p(from29(prev[i * ss_prev + 1]));
        val[i] = a + rr * (b - a);
        final_vals[i] = val[i];
      } else {
        val[i] = Fr::zero();
      }
    }
    *evaluation = sop_eval_final<K>(spg, h.nmono, val);
  }
  // absorb the last challenge bytes
  if (pending && tid < 64) b3_hash_quad(pend, 80, ro.st->state, 8);
}

// ---------------------------------------------------------------------------
// Slice tail (replaces k_sc_tail whenever a block's slice fits its LDS): the
// rounds j0..nvars-1 in ONE launch of G blocks (one per CU), block b OWNING
// the contiguous entries [b S, (b+1) S) of the round-j0 table (S = 2^(nvars -
// j0) / G per slot).  The fold pairs adjacent entries, so block b's slice of
// round j+1 is the fold of its own slice of round j: after the one HBM load
// of the first round the tables never leave the block's LDS, and nothing but
// the per-round sums crosses blocks (partial rows + grid barrier, then every
// block runs the identical transcript step).  When a slice is down to one
// pair, each block folds it to one entry per slot, writes it to HBM, and
// after one more barrier block 0 gathers the G entries and finishes the last
// log2(G) rounds alone (the table again in LDS).  The deferred absorb of the
// previous challenge runs on the last wave beside the other waves' evaluation.
// ---------------------------------------------------------------------------
#ifndef QG_SL_BLOCK
#define QG_SL_BLOCK 256
#endif
static constexpr int SL_BLOCK = QG_SL_BLOCK;
// entries per slot of a block's slice in the first tail round (LDS: K slots x
// 1.5 x SL_SMAX entries of 36 B: the slice and its half-size fold)
QG_HD constexpr uint32_t sl_smax(int K) { return K <= 4 ? 256u : 128u; }

template <int K, int NP>
__global__ void __launch_bounds__(SL_BLOCK)
    k_sc_slice(TablePtrs tp0, TablePtrs gat, const SopDev* __restrict__ spg, SopHdr h,
               uint32_t nvars, uint32_t j0, int fold0, int pending0, RoundOut ro,
               uint64_t* __restrict__ acc_j0, uint32_t* __restrict__ bar8,
               uint64_t* __restrict__ acc64, Fr* __restrict__ final_vals,
               Fr* __restrict__ evaluation) {
  constexpr uint32_t SMAX = sl_smax(K);
  __shared__ SopLds<NP> sp;
  __shared__ R29 Fbuf[K * SMAX * 3 / 2];
  __shared__ R29 red[(SL_BLOCK / 64) * NP];
  __shared__ R29 res[NP];
  __shared__ FinSmem fs;
  __shared__ uint32_t st[8];
  __shared__ uint32_t pend[32];
  __shared__ uint64_t lsum[NP * 9];
  const uint32_t tid = threadIdx.x, blk = blockIdx.x;
  const uint32_t nslots = h.nslots, np = h.np;
  const uint32_t t = tid % NP;
  const bool last_wave = tid >= SL_BLOCK - 64;
  // per-round limb accumulators of rounds > j0: [round - j0 - 1][shard 8][NP][9],
  // zeroed here by block 0 before it meets the others at round j0's barrier
  // (round j0 adds into acc_j0, already clear)
  constexpr uint32_t ACC_R = 8 * NP * 9;
  if (blk == 0)
    for (uint32_t i = tid; i < (nvars - j0 - 1) * ACC_R; i += SL_BLOCK)
      __hip_atomic_store((gu64*)(acc64 + i), (uint64_t)0, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  uint32_t arrived = 0;                          // cumulative barrier arrivals
  uint32_t G = gridDim.x;                        // blocks holding a slice this round
  uint32_t S = (1u << (nvars - j0)) / G;         // entries per slot of this block's slice
  sop_load<NP>(sp, spg, h, true);
  if (tid < 8) st[tid] = ro.st->state[tid];
  if (tid < 32) pend[tid] = (pending0 && tid < 20) ? ro.st->pend[tid] : 0u;
  R29 r = R29::zero();
  if (fold0) {
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = ro.st->r29[i];
  }
  R29* cur = Fbuf;                // slot stride S
  R29* nxt = Fbuf + K * SMAX;     // slot stride S / 2
  // the block's slice of the round-j0 table (folded from the source by r_{j0-1})
  for (uint32_t it = tid; it < nslots * S; it += SL_BLOCK) {
    const uint32_t s = it / S, e = it % S;
    const size_t idx = (size_t)blk * S + e;
    R29 v;
    if (fold0) {
      const Fr* src = tp0.src[s] + 2 * idx;
      const R29 x0 = to29(src[0]), x1 = to29(src[1]);
      v = red2p29<FrP>(add29(x0, mul29(sub29(x1, x0), r)));
    } else {
      v = to29(tp0.src[s][idx]);
    }
    cur[s * S + e] = v;
  }
  int pending = pending0;
  __syncthreads();
  for (uint32_t j = j0; j < nvars; j++) {
    if (blk == 0) SC_TR(16 * j + 0);
    // ---- evaluate round j on the slice: thread (pair, point) items; the last
    // wave absorbs the previous challenge instead when one is pending
    // a round that regroups (below) publishes its slice before the barrier
    const bool regroup = G > 1 && S <= SMAX / 8;
    if (regroup)
      for (uint32_t it = tid; it < nslots * S; it += SL_BLOCK) {
        const uint32_t s = it / S, e = it % S;
        st_sc1(gat.dst[s] + (size_t)blk * S + e, from29(cur[s * S + e]));
      }
    const uint32_t ne = pending ? SL_BLOCK - 64 : SL_BLOCK;
    if (pending && last_wave) b3_hash_quad(pend, 80, st, 8);
    R29 acc = R29::zero();
    const uint32_t items = (S / 2) * NP;
    if (tid < ne)
      for (uint32_t it = tid; it < items; it += ne)
        if (t < np) tail_eval<NP>(cur, S, sp, h, it / NP, t, acc);
    if (blk == 0) SC_TR(16 * j + 1);
    tail_reduce<NP>(acc, std::min(items, ne), np, red, res);
    if (blk == 0) SC_TR(16 * j + 7);
    if (G > 1) {
      // limbs of the block sums added into this round's accumulator shard
      // (agent-scope u64 atomics at the memory side), one sharded barrier, then
      // every block fetches the 8 shards with returning atomics and rebuilds
      // the sums: no partial rows, one memory round trip.  Round j0 uses the
      // big rounds' cleared slot (shard stride 16 x 9), later rounds acc64.
      uint64_t* ar = j == j0 ? acc_j0 : acc64 + (size_t)(j - j0 - 1) * ACC_R;
      const uint32_t ss = j == j0 ? 16 * 9 : NP * 9;
      if (tid < np * 9)
        __hip_atomic_fetch_add((gu64*)(ar + (blk & 7) * ss + tid),
                               (uint64_t)res[tid / 9].l[tid % 9], __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      arrived += G;
      grid_barrier8(bar8, arrived, &ro.st->err);
      if (blk == 0) SC_TR(16 * j + 8);
      if (tid < np * 9) {
        uint64_t v[8], a = 0;
#pragma unroll
        for (int x = 0; x < 8; x++)
          v[x] = __hip_atomic_fetch_add((gu64*)(ar + x * ss + tid), (uint64_t)0,
                                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int x = 0; x < 8; x++) a += v[x];
        lsum[tid] = a;
      }
      __syncthreads();
      if (tid < np) res[tid] = limbsum29(lsum + 9 * tid);
      __syncthreads();
    }
    if (blk == 0) SC_TR(16 * j + 2);
    finish_core<NP>(sp, np, res, ro, j, fs, st, pend, nullptr, blk == 0 ? 16 * j : 4096, blk == 0,
                    true);
    __syncthreads();
    r = fs.r;
    pending = 1;
    if (j + 1 == nvars) break;  // S == 2, G == 1: the final fold below
    if (regroup) {
      // f blocks' round-j slices (published before the barrier) become one
      // block's round-(j+1) slice, folded on the load; the other blocks retire.
      // Fewer blocks: a cheaper barrier and fewer partial rows per round.
      const uint32_t f = std::min<uint32_t>(G, 2 * SMAX / S);
      const uint32_t G2 = G / f;
      if (blk >= G2) return;
      const uint32_t S2 = f * S / 2;
      for (uint32_t it = tid; it < nslots * S2; it += SL_BLOCK) {
        const uint32_t s = it / S2, e = it % S2;
        const Fr* src = gat.dst[s] + (size_t)blk * f * S + 2 * e;
        const R29 x0 = to29(ld_sc1(src)), x1 = to29(ld_sc1(src + 1));
        Fbuf[s * S2 + e] = red2p29<FrP>(add29(x0, mul29(sub29(x1, x0), r)));
      }
      S = S2;
      G = G2;
      cur = Fbuf + K * SMAX;  // swapped below: cur = Fbuf (S2 <= SMAX), nxt = the second array
      nxt = Fbuf;
    } else {
      // fold the slice by r_j into the other array
      const uint32_t h2 = S / 2;
      for (uint32_t it = tid; it < nslots * h2; it += SL_BLOCK) {
        const uint32_t s = it / h2, e = it % h2;
        const R29 x0 = cur[s * S + 2 * e], x1 = cur[s * S + 2 * e + 1];
        nxt[s * h2 + e] = red2p29<FrP>(add29(x0, mul29(sub29(x1, x0), r)));
      }
      S = h2;
    }
    R29* tmp = cur;
    cur = nxt;
    nxt = tmp;
    __syncthreads();
  }
  // final fold with r_{n-1} on the 32-bit path: one pair per slot left in cur (block 0)
  if (tid == 0) {
    const Fr rr = fs.r256;
    Fr val[K];
#pragma unroll
    for (int i = 0; i < K; i++) {
      if ((uint32_t)i < nslots) {
        const Fr a = lt_p(from29(cur[i * 2])), b = lt_p(from29(cur[i * 2 + 1]));
        val[i] = a + rr * (b - a);
        final_vals[i] = val[i];
      } else {
        val[i] = Fr::zero();
      }
    }
    *evaluation = sop_eval_final<K>(spg, h.nmono, val);
  }
  // absorb the last challenge bytes
  if (pending && tid < 64) b3_hash_quad(pend, 80, ro.st->state, 8);
}

// ---------------------------------------------------------------------------
// Generic expressions: everything the compiled fast path does not take (more
// than 8 tables, degree above 15, a monomial expansion beyond 256 / 1024
// terms, or one that does not expand at all).  The postfix program itself is
// interpreted per (pair, point) — the reference's evaluate_expr_poly tree walk
// (virtual_polynomial.rs:300-320) on point values instead of polynomials —
// with every value in the R = 2^261 domain (inputs converted on load), so
// Add / Mul need no scale bookkeeping.  Per round: a fold kernel (all slots,
// r_{j-1}), the evaluation kernel (per-block per-point partial rows), a
// one-block row sum; the transcript step runs on the host (one round trip
// per round: this path is for coverage, the fast path stays on the device).
// ---------------------------------------------------------------------------
static constexpr int GEN_NPMAX = 32;  // points per round (syntactic degree <= 31)
static constexpr int GEN_STACK = 32;  // interpreter stack (postfix depth)

struct GenOp {
  uint32_t op, arg;  // QG_OP_*; INPUT: used-slot index; CONST: constant index
};

// postfix interpreter; load(slot) returns the slot's value in the 2^261 domain
template <class Load>
__device__ __forceinline__ R29 gen_interp(const GenOp* __restrict__ ops, uint32_t len,
                                          const L9* __restrict__ consts29, Load load) {
  R29 stk[GEN_STACK];
  uint32_t sp = 0;
  for (uint32_t i = 0; i < len; i++) {
    const GenOp o = ops[i];
    if (o.op == QG_OP_INPUT) {
      stk[sp++] = load(o.arg);
    } else if (o.op == QG_OP_CONST) {
      stk[sp++] = R29::from_l9(consts29[o.arg]);
    } else {
      const R29 b = stk[--sp], a = stk[--sp];
      stk[sp++] = o.op == QG_OP_ADD ? red2p29(add29(a, b)) : mul29(a, b);
    }
  }
  return stk[0];
}

template <int NPP>
__global__ void __launch_bounds__(256)
    k_gen_eval(const Fr* const* __restrict__ tabs, size_t npairs, uint32_t np,
               const GenOp* __restrict__ ops, uint32_t len, const L9* __restrict__ consts29,
               const L9* __restrict__ t29, Fr* __restrict__ partial) {
  __shared__ R29 red[4 * NPP];
  __shared__ R29 res[NPP];
  constexpr uint32_t PB = 256 / NPP;
  const uint32_t tid = threadIdx.x, t = tid % NPP, pl = tid / NPP;
  const R29 to261 = R29::from_l9(F29P<FrP>::TO261);
  R29 acc = R29::zero();
  for (size_t base = (size_t)blockIdx.x * PB; base < npairs; base += (size_t)gridDim.x * PB) {
    const size_t p = base + pl;
    if (p >= npairs || t >= np) continue;
    const R29 tt = R29::from_l9(t29[t]);
    const R29 v = gen_interp(ops, len, consts29, [&](uint32_t s) {
      const Fr* tb = tabs[s];
      const R29 lo = to29(tb[2 * p]), hi = to29(tb[2 * p + 1]);
      // lo + t (hi - lo) in arkworks form (< 2p), then into the 2^261 domain
      return mul29(red6p(add29(lo, mul29(sub29(hi, lo), tt))), to261);
    });
    acc = red2p29(add29(acc, v));
  }
  block_reduce_pts<NPP>(acc, np, red, res);
  if (tid < NPP) partial[(size_t)blockIdx.x * NPP + tid] = from29(canon29(tid < np ? res[tid] : R29::zero()));
}

// out[x] = h(x) for every row (canonical Montgomery words)
__global__ void __launch_bounds__(256)
    k_gen_table(const Fr* const* __restrict__ tabs, size_t n, const GenOp* __restrict__ ops,
                uint32_t len, const L9* __restrict__ consts29, Fr* __restrict__ out) {
  const size_t x = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= n) return;
  const R29 to261 = R29::from_l9(F29P<FrP>::TO261);
  const R29 v = gen_interp(ops, len, consts29,
                           [&](uint32_t s) { return mul29(to29(tabs[s][x]), to261); });
  out[x] = from29(canon29(mul29(v, R29::from_l9(F29P<FrP>::TO256))));
}

// one block: per-point sums of the partial rows, 2^261 domain -> Montgomery
// (x 2^256) words for the host's interpolation
template <int NPP>
__global__ void __launch_bounds__(256)
    k_gen_rows(const Fr* __restrict__ partial, uint32_t nrows, uint32_t np, Fr* __restrict__ out) {
  __shared__ R29 red[4 * NPP];
  __shared__ R29 res[NPP];
  sum_rows29<NPP>(partial, nrows, np, red, res);
  if (threadIdx.x < np)
    out[threadIdx.x] = from29(canon29(mul29(res[threadIdx.x], R29::from_l9(F29P<FrP>::TO256))));
}

// fold every slot by r (x 2^261 in st->r29): dst[s][q] = x0 + r (x1 - x0) (< 2p)
__global__ void k_gen_fold(const Fr* const* __restrict__ src, Fr* const* __restrict__ dst,
                           uint32_t nslots, size_t nq, const ScState* __restrict__ st) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nq * nslots) return;
  const uint32_t s = (uint32_t)(i / nq);
  const size_t q = i % nq;
  R29 r;
#pragma unroll
  for (int k = 0; k < 9; k++) r.l[k] = st->r29[k];
  const R29 x0 = to29(src[s][2 * q]), x1 = to29(src[s][2 * q + 1]);
  dst[s][q] = from29(red6p(add29(x0, mul29(sub29(x1, x0), r))));
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

// host helpers on plain integers (< p)
static Fr plain_mul(const Fr& x, const Fr& y) { return from_mont(to_mont(x) * to_mont(y)); }
static Fr from_u64_plain(uint64_t v) {
  Fr r = Fr::zero();
  r.v[0] = (uint32_t)v;
  r.v[1] = (uint32_t)(v >> 32);
  return r;
}
static L9 l9_of(const Fr& x) {
  const R29 t = to29(x);
  L9 r{};
  for (int i = 0; i < 9; i++) r.v[i] = t.l[i];
  return r;
}

// inverse Vandermonde on nodes 0..np-1: coefficient t of sum_u L_u(X) ev[u] is
// sum_u V[t][u] ev[u]; out_m[t*16+u] = V (Montgomery), out_c = V (plain)
static void build_vinv(uint32_t np, Fr* out_m, Fr* out_c) {
  for (uint32_t i = 0; i < 16 * 16; i++) out_m[i] = out_c[i] = Fr::zero();
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
    for (uint32_t i = 0; i < np; i++) {
      out_m[i * 16 + j] = poly[i] * dinv;
      out_c[i * 16 + j] = from_mont(out_m[i * 16 + j]);
    }
  }
}

// Compiled programs are cached by their exact bytes (the device image carries
// the inverse Vandermonde, whose host construction costs field inversions).
struct ScProgram {
  uint64_t id = 0;  // unique per compiled program (device-copy memo key)
  SopDev img;
  SopHdr hdr;
  uint32_t nused = 0;
  std::vector<uint32_t> used;
  uint32_t width = 0;  // syntactic degree + 1 (proof row width)
};

static std::mutex g_prog_mu;
static std::map<std::string, std::shared_ptr<const ScProgram>> g_prog_cache;

static std::shared_ptr<const ScProgram> get_program(const qg_expr_op* prog, size_t prog_len,
                                                    const uint64_t* consts, size_t nconsts,
                                                    uint32_t ntables) {
  std::string key((const char*)&ntables, 4);
  key.append((const char*)prog, prog_len * sizeof(qg_expr_op));
  key.push_back('|');
  if (nconsts) key.append((const char*)consts, nconsts * 32);
  {
    std::lock_guard<std::mutex> lk(g_prog_mu);
    auto it = g_prog_cache.find(key);
    if (it != g_prog_cache.end()) return it->second;
  }
  static std::atomic<uint64_t> next_id{1};
  auto p = std::make_shared<ScProgram>();
  p->id = next_id++;
  p->width = expr_degree(prog, prog_len) + 1;
  SopProgram sp = compile_program(prog, prog_len, consts, nconsts, ntables);
  QG_CHECK(sp.mono_len.size() <= (size_t)SOP_MAXM && sp.fac.size() <= (size_t)SOP_MAXF,
           QG_ERR_UNSUPPORTED, "expression too large");
  QG_CHECK(sp.used.size() <= 8, QG_ERR_UNSUPPORTED, "expression uses more than 8 tables");
  QG_CHECK(sp.degree <= 15, QG_ERR_UNSUPPORTED, "expression degree above 15");
  const uint32_t np = sp.degree + 1;
  QG_CHECK(np <= p->width, QG_ERR_ASSERT, "degree bookkeeping");
  SopDev& d = p->img;
  memset(&d, 0, sizeof(SopDev));
  d.nmono = (uint32_t)sp.mono_len.size();
  d.nslots = (uint32_t)sp.used.size();
  d.np = np;
  d.nfac = (uint32_t)sp.fac.size();
  // scale bookkeeping of the 29-bit evaluation (see SopDev): e = 5 (dmax - 1)
  const int dmax = (int)sp.degree, e = 5 * (dmax - 1);
  for (size_t m = 0; m < sp.mono_len.size(); m++) {
    const int dm = (int)sp.mono_len[m];
    d.mono_len[m] = (uint8_t)dm;
    d.is_one[m] = sp.is_one[m];
    d.coeff[m] = sp.coeff[m];
    const Fr c = from_mont(sp.coeff[m]);
    const uint32_t k = dm == 0 ? (uint32_t)(256 - e) : (uint32_t)(261 - 5 * (dmax - dm));
    d.c29[m] = l9_of(plain_mul(c, pow2_mod_plain<FrP>(k)));
    d.skip29[m] = (dm == dmax && dm >= 2 && sp.is_one[m]) ? 1 : 0;
  }
  for (size_t f = 0; f < sp.fac.size(); f++) d.fac[f] = (uint8_t)sp.fac[f];
  {
    Fr vm[16 * 16], vc[16 * 16];
    build_vinv(np, vm, vc);  // vc: plain inverse-Vandermonde entries
    const Fr sm = pow2_mod_plain<FrP>((uint32_t)(261 + e)), sc = pow2_mod_plain<FrP>((uint32_t)(5 + e));
    for (uint32_t i = 0; i < 16 * 16; i++) {
      d.vm29[i] = l9_of(plain_mul(vc[i], sm));
      d.vc29[i] = l9_of(plain_mul(vc[i], sc));
    }
  }
  for (uint32_t t = 0; t < 16; t++)
    d.t29[t] = l9_of(plain_mul(from_u64_plain(t), pow2_mod_plain<FrP>(261)));
  d.cr29[0] = l9_of(pow2_mod_plain<FrP>(522));
  d.cr29[1] = l9_of(pow2_mod_plain<FrP>(778));
  d.cr29[2] = l9_of(pow2_mod_plain<FrP>(517));
  d.cr29[3] = l9_of(pow2_mod_plain<FrP>(773));
  d.cs29 = l9_of(pow2_mod_plain<FrP>((uint32_t)(517 - e)));
  bool pure = d.nmono == 1 && sp.is_one[0] && sp.mono_len[0] == d.nslots && d.nslots >= 2 &&
              d.nslots == sp.degree;
  for (uint32_t f = 0; pure && f < d.nfac; f++) pure = sp.fac[f] == f;
  p->hdr = {d.nmono, d.nslots, np, pure ? SOP_PURE : 0u};
  p->used = sp.used;
  p->nused = (uint32_t)sp.used.size();
  std::lock_guard<std::mutex> lk(g_prog_mu);
  if (g_prog_cache.size() >= 256) g_prog_cache.clear();
  g_prog_cache[key] = p;
  return p;
}


// Co-residency guard of a grid-barrier launch: the grid must not exceed what
// the device holds at once (occupancy API x CUs, one block per CU margin kept
// for the gfx950 SGPR admission rule of MI355X_MICROARCH.md "Residency").
// Queried once per context and kernel instantiation.
template <int K, int NP, bool SLICE = false>
static unsigned persist_grid_cap(qg_ctx* ctx, size_t cus) {
  const std::string key = std::string(SLICE ? "slice_occ_" : "persist_occ_") + std::to_string(K) +
                          "_" + std::to_string(NP);
  auto it = ctx->memo.find(key);
  int occ = 0;
  if (it == ctx->memo.end()) {
    const void* fn = SLICE ? reinterpret_cast<const void*>(&k_sc_slice<K, NP>)
                           : reinterpret_cast<const void*>(&k_sc_tail<K, NP>);
    QG_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, SLICE ? SL_BLOCK : TAIL_BLOCK, 0));
    ctx->memo[key] = std::to_string(occ);
  } else {
    occ = std::stoi(it->second);
  }
  QG_CHECK(occ >= 1, QG_ERR_DEVICE, "persistent sumcheck kernel cannot be resident");
  // bpc blocks per CU (QG_SC_TAIL_BPC, default 1), never more than the
  // occupancy answer minus one: a spare block slot per CU keeps the barrier
  // safe next to other kernels' blocks and under the gfx950 SGPR admission
  // rule (MI355X_MICROARCH.md "Residency")
  static const int bpc_env = [] {
    const char* e = getenv("QG_SC_TAIL_BPC");
    return e ? std::max(1, atoi(e)) : 1;
  }();
  const int bpc = std::max(1, std::min(bpc_env, occ - 1));
  return (unsigned)std::max<size_t>(1, cus * (size_t)bpc);
}

// io header: ScState | per-round barrier counters (nvars + 2) | 8 barrier
// shards of the slice tail, one 128-B line each | challenges ...
static size_t sumcheck_o_bar8(uint32_t nvars) {
  return (sizeof(ScState) + sizeof(uint32_t) * (nvars + 2) + 127) & ~(size_t)127;
}
static uint32_t* sumcheck_bar8(uint32_t* bar, uint32_t nvars) {
  uint8_t* io = reinterpret_cast<uint8_t*>(bar) - sizeof(ScState);
  return reinterpret_cast<uint32_t*>(io + sumcheck_o_bar8(nvars));
}
// big-round limb accumulators (k_sc_big): [shard 8][16 points][9 limbs] u64;
// round 0's in the io header after the barrier shards (zeroed per call),
// round 1's in scratch; each round's last block clears the next round's
static constexpr size_t SC_BACC_BYTES = 8 * 16 * 9 * sizeof(uint64_t);
static size_t sumcheck_o_bacc0(uint32_t nvars) { return sumcheck_o_bar8(nvars) + 8 * 128; }
static uint64_t* sumcheck_bacc0(uint32_t* bar, uint32_t nvars) {
  uint8_t* io = reinterpret_cast<uint8_t*>(bar) - sizeof(ScState);
  return reinterpret_cast<uint64_t*>(io + sumcheck_o_bacc0(nvars));
}

// The slice tail (k_sc_slice): G blocks, a power of two <= min(one per CU,
// SMAX) so block 0 can gather one entry per block, each owning <= SMAX entries
// per slot.  QG_SC_OLD_TAIL=1 keeps the streaming k_sc_tail (A/B runs).
template <int K, int NP>
static size_t slice_gmax(qg_ctx* ctx, size_t cus) {
  const char* off = getenv("QG_SC_OLD_TAIL");  // read per call: tests toggle it in-process
  if (off && atoi(off) != 0) return 0;
  const size_t gm = std::min<size_t>(persist_grid_cap<K, NP, true>(ctx, cus), sl_smax(K));
  size_t G = 1;
  while (G * 2 <= gm) G *= 2;
  return G;
}

// largest round table (entries per slot) the slice tail can start from
template <int K, int NP>
static uint32_t slice_tail_log(qg_ctx* ctx, size_t cus) {
  const size_t g = slice_gmax<K, NP>(ctx, cus);
  if (!g) return 0;
  uint32_t l = 0;
  while (((size_t)1 << (l + 1)) <= g * sl_smax(K)) l++;
  return l;
}

// launches k_sc_slice for rounds j0.. when a block's slice fits its LDS;
// false: the caller launches k_sc_tail.
template <int K, int NP>
static bool launch_slice_tail(qg_ctx* ctx, size_t cus, TablePtrs t0, const SopDev* d_sp, SopHdr h,
                              uint32_t nvars, uint32_t j0, int fold0, int pending0, RoundOut ro,
                              uint32_t* bar, uint64_t* acc_j0, Fr* d_final, Fr* d_eval) {
  const size_t gm = slice_gmax<K, NP>(ctx, cus);
  if (!gm) return false;
  const size_t n0 = (size_t)1 << (nvars - j0);
  size_t G = 1;
  while (G * 2 <= gm && G * 2 <= n0 / 2) G *= 2;
  if (n0 / G > sl_smax(K)) return false;
  uint64_t* acc64 = ctx->scratch_as<uint64_t>("sc_sacc", (size_t)std::max<uint32_t>(1, nvars - j0) * 8 * NP * 9);
  // the 8 barrier shards follow the per-round counters (zeroed by the per-call
  // header copy): sumcheck_bar8
  uint32_t* bar8 = sumcheck_bar8(bar, nvars);
  // regroup area: the round table published by the blocks (<= n0 entries per slot)
  const uint32_t ns = std::max<uint32_t>(h.nslots, 1u);
  Fr* sg = ctx->scratch_as<Fr>("sc_sgat", (size_t)ns * n0);
  TablePtrs gat{};
  for (uint32_t i = 0; i < 8; i++) gat.dst[i] = i < h.nslots ? sg + (size_t)i * n0 : nullptr;
  hipLaunchKernelGGL((k_sc_slice<K, NP>), dim3((unsigned)G), dim3(SL_BLOCK), 0, ctx->stream, t0,
                     gat, d_sp, h, nvars, j0, fold0, pending0, ro, acc_j0, bar8, acc64, d_final,
                     d_eval);
  QG_LAUNCH_CHECK();
  return true;
}

// thread-per-pair round kernel (k_sc_big) for product expressions and for
// expressions of <= 4 slots at degree <= 3; false: use the staged k_sc_round
static unsigned sc_big_blocks(qg_ctx* ctx, size_t npairs) {
  static int ov = [] {
    const char* e = getenv("QG_SC_BIG_BLOCKS");
    return e ? atoi(e) : 0;
  }();
  size_t cap = ov > 0 ? (size_t)ov : (size_t)2 * ctx->num_cus();  // measured best (256 / 512 / 2048 blocks at 2^20: 0.289 / 0.264 / 0.333 ms)
  cap = std::min<size_t>(cap, SC_MAX_BLOCKS);
  return (unsigned)std::max<size_t>(1, std::min<size_t>(cap, div_up(npairs, SC_BLOCK)));
}

// returns -1 when the staged k_sc_round must run instead, else the skip0 flag used
template <int K, int NP>
static int launch_big(qg_ctx* ctx, const std::vector<const Fr*>& src, Fr* X, Fr* Y, size_t N,
                       uint32_t j, const SopDev* d_sp, SopHdr h, size_t npairs, RoundOut ro,
                       int pending, Fr* loc, uint64_t* a0, uint64_t* a1, uint32_t* bar8) {
  // rounds j >= 1: h(0) = h_{j-1}(r_{j-1}) - h(1), exact by construction (the
  // folded table's pair sums ARE the previous message at r); round 0 evaluates
  // every point, so a wrong caller claim still yields the reference's bytes.
  // QG_SC_NO_SKIP0=1 evaluates t = 0 in every round (A/B runs).
  static const bool no_skip0 = getenv("QG_SC_NO_SKIP0") != nullptr;
  const int skip0 = (j >= 1 && h.np >= 2 && !no_skip0) ? 1 : 0;
  if (sc_use_staged() || NP > 4) return -1;
  const bool pure = (h.pad & SOP_PURE) != 0;
  if (!pure && K > 4) return -1;
  AllBufs tb{};
  for (uint32_t i = 0; i < 8; i++) tb.in.src[i] = i < src.size() ? src[i] : nullptr;
  tb.X = X;
  tb.Y = Y;
  tb.capX = N / 2;
  tb.capY = std::max<size_t>(1, N / 4);
  const unsigned blocks = sc_big_blocks(ctx, npairs);
  // QG_SC_WPE=4: the product sweep compiled for 4 waves per SIMD (<= 128 VGPRs,
  // spills; tuning.  3 waves measured too: 0.214 -> 0.288 ms of big rounds,
  // profiles/r04_sumcheck_wpe_blocks_ab.txt)
  static const bool wpe4 = getenv("QG_SC_WPE") != nullptr;
  if (pure && wpe4)
    hipLaunchKernelGGL((k_sc_big<K, 4, true, 4>), dim3(blocks), dim3(SC_BLOCK), 0,
                       ctx->stream, tb, j, d_sp, h, npairs, ro, pending, loc, skip0, (j & 1) ? a1 : a0,
                       (j & 1) ? a0 : a1, bar8);
  else if (pure)
    hipLaunchKernelGGL((k_sc_big<K, 4, true>), dim3(blocks), dim3(SC_BLOCK), 0, ctx->stream,
                       tb, j, d_sp, h, npairs, ro, pending, loc, skip0, (j & 1) ? a1 : a0,
                       (j & 1) ? a0 : a1, bar8);
  else
    hipLaunchKernelGGL((k_sc_big<4, 4, false>), dim3(blocks), dim3(SC_BLOCK), 0, ctx->stream,
                       tb, j, d_sp, h, npairs, ro, pending, loc, skip0, (j & 1) ? a1 : a0,
                       (j & 1) ? a0 : a1, bar8);
  QG_LAUNCH_CHECK();
  return skip0;
}

// returns the first round of the persistent tail (its coefficient rows are
// canonical words: k_sc_tail's finish_core canon_out)
template <int K, int NP>
static uint32_t run_rounds(qg_ctx* ctx, uint32_t nvars, const std::vector<const Fr*>& src,
                       const SopDev* d_sp, SopHdr h, RoundOut ro, uint32_t* bar, Fr* d_final,
                       Fr* d_eval) {

  const uint32_t nslots = h.nslots;
  const size_t N = (size_t)1 << nvars;
  // ping-pong scratch: X holds N/2 per slot, Y holds N/4 per slot
  Fr* X = ctx->scratch_as<Fr>("sc_x", std::max<size_t>(1, (N / 2) * nslots));
  Fr* Y = ctx->scratch_as<Fr>("sc_y", std::max<size_t>(1, (N / 4) * nslots));
  Fr* partial = ctx->scratch_as<Fr>("sc_partial", (size_t)SC_MAX_BLOCKS * NP);
  uint64_t* a0 = sumcheck_bacc0(bar, nvars);
  uint64_t* a1 = reinterpret_cast<uint64_t*>(ctx->scratch_as<uint8_t>("sc_bacc1", SC_BACC_BYTES));
  uint32_t* bar8 = sumcheck_bar8(bar, nvars);
  // the staged round kernel does not clear the next accumulator slot: the
  // tail's first slot is then cleared here when it is the scratch one
  bool staged = false;
  auto clear_tail_slot = [&](uint32_t j0) {
    if (staged && (j0 & 1)) QG_HIP(hipMemsetAsync(a1, 0, SC_BACC_BYTES, ctx->stream));
  };
  TablePtrs cur{};
  for (uint32_t i = 0; i < 8; i++) cur.src[i] = i < src.size() ? src[i] : nullptr;
  auto bufs = [&](Fr* base, size_t per) {
    TablePtrs t{};
    for (uint32_t i = 0; i < 8; i++) t.dst[i] = i < nslots ? base + per * i : nullptr;
    return t;
  };
  TablePtrs tX = bufs(X, N / 2), tY = bufs(Y, std::max<size_t>(1, N / 4));
  int fold = 0, pending = 0;
  uint32_t j = 0;
  int parity = 0;  // next destination: 0 -> X, 1 -> Y
  // QG_SC_PERS_LOG overrides where the persistent tail takes over (tuning)
  static const int pers_log = [] {
    const char* e = getenv("QG_SC_PERS_LOG");
    return e ? atoi(e) : PERS_LOG;
  }();
  {
    QgTimed tm(ctx, "sumcheck_round");
    // the slice tail starts once a round's table fits the blocks' LDS slices
    const uint32_t sl = slice_tail_log<K, NP>(ctx, ctx->num_cus());
    const int plog = sl ? std::min<int>(pers_log, (int)sl) : pers_log;
    for (; j < nvars; j++) {
      const size_t table = N >> j;  // entries per table evaluated in round j
      if (table <= ((size_t)1 << plog)) break;
      const size_t npairs = table / 2;
      TablePtrs tp = cur;
      if (fold) {
        const TablePtrs& d = parity ? tY : tX;
        for (int i = 0; i < 8; i++) tp.dst[i] = d.dst[i];
      }
      if (launch_big<K, NP>(ctx, src, X, Y, N, j, d_sp, h, npairs, ro, pending, nullptr, a0, a1,
                            bar8) < 0) {
        hipLaunchKernelGGL((k_sc_round<K, NP>), dim3(sc_round_blocks(ctx, npairs)), dim3(SC_BLOCK),
                           0, ctx->stream, tp, d_sp, h, npairs, fold, ro, j, pending, partial,
                           (Fr*)nullptr);
        staged = true;
      }
      QG_LAUNCH_CHECK();
      if (fold) {
        for (int i = 0; i < 8; i++) cur.src[i] = tp.dst[i];
        parity ^= 1;
      }
      fold = 1;
      pending = 1;
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
    // round j's accumulator slot was cleared by the last big round (or the
    // per-call header when there is none)
    clear_tail_slot(j);
    if (!launch_slice_tail<K, NP>(ctx, ctx->num_cus(), t0, d_sp, h, nvars, j, fold, pending, ro,
                                  bar, (j & 1) ? a1 : a0, d_final, d_eval)) {
      // persistent launch: one block per CU at most (co-residency for the grid
      // barrier), fewer when the first persistent round has fewer pair groups
      const size_t PB = tail_pb(h.nslots, NP);
      const size_t pairs0 = (N >> j) / 2;
      const unsigned grid = (unsigned)std::max<size_t>(
          1, std::min<size_t>(persist_grid_cap<K, NP>(ctx, ctx->num_cus()), (pairs0 + PB - 1) / PB));
      Fr* ppart = ctx->scratch_as<Fr>("sc_ppartial", (size_t)2 * grid * NP);
      hipLaunchKernelGGL((k_sc_tail<K, NP>), dim3(grid), dim3(TAIL_BLOCK), 0, ctx->stream, t0,
                         bufA, bufB, d_sp, h, nvars, j, fold, pending, ro, ppart, bar, d_final,
                         d_eval);
      QG_LAUNCH_CHECK();
    }
  }
  return j;
}

// gathered [rank][slot][e] (S entries per rank and slot) -> per-slot tables
// [slot][rank * S + e]: the rank is the high index bits
__global__ void k_sc_gather_tables(const Fr* __restrict__ in, uint32_t world, uint32_t nslots,
                                   size_t S, Fr* __restrict__ out) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t total = (size_t)world * nslots * S;
  if (idx >= total) return;
  const size_t e = idx % S, sl = (idx / S) % nslots, rk = idx / (S * nslots);
  out[sl * world * S + rk * S + e] = in[idx];
}

// Sharded rounds: this rank holds the block of every table whose
// high log2(world) index bits equal its rank.  The large rounds 0..js-1 pair
// local entries only: one allgather of the (d+1) round sums per round, then
// every rank runs the identical device transcript (k_sc_finish).  Once the
// folded tables are small (global size <= 2^(SC_GATHER_LOG)) every rank
// allgathers its block and runs the remaining rounds redundantly in the
// single-GPU persistent kernel — no per-round collective on the
// latency-bound tail (which does not shrink with more GPUs anyway).
static constexpr uint32_t SC_GATHER_LOG = 16;

template <int K, int NP>
static uint32_t run_rounds_dist(qg_ctx* ctx, uint32_t nvars, const std::vector<const Fr*>& src,
                            const SopDev* d_sp, SopHdr h, RoundOut ro, uint32_t* bar, Fr* d_final,
                            Fr* d_eval) {
  const uint32_t nslots = h.nslots;
  const uint32_t world = (uint32_t)ctx->world;
  uint32_t lw = 0;
  while ((1u << lw) < world) lw++;
  QG_CHECK((1u << lw) == world, QG_ERR_INVALID, "sharded sumcheck needs a power-of-two world");
  QG_CHECK(nvars > lw, QG_ERR_INVALID, "sharded sumcheck needs nvars > log2(world)");
  const uint32_t m = nvars - lw;
  const size_t NL = (size_t)1 << m;
  // sharded rounds: until the source tables of round js (folded through
  // r_{js-2}, global size 2^(nvars - js + 1)) fit the gather size; at most m
  // (local tables of 2 entries)
  uint32_t js = nvars + 1 > SC_GATHER_LOG ? nvars + 1 - SC_GATHER_LOG : 0;
  if (js > m) js = m;
  Fr* X = ctx->scratch_as<Fr>("sc_x", std::max<size_t>(1, (NL / 2) * std::max(nslots, 1u)));
  Fr* Y = ctx->scratch_as<Fr>("sc_y", std::max<size_t>(1, (NL / 4) * std::max(nslots, 1u)));
  Fr* partial = ctx->scratch_as<Fr>("sc_partial", (size_t)SC_MAX_BLOCKS * NP);
  uint64_t* a0 = sumcheck_bacc0(bar, nvars);
  uint64_t* a1 = reinterpret_cast<uint64_t*>(ctx->scratch_as<uint8_t>("sc_bacc1", SC_BACC_BYTES));
  uint32_t* bar8 = sumcheck_bar8(bar, nvars);
  // the staged round kernel does not clear the next accumulator slot: the
  // tail's first slot is then cleared here when it is the scratch one
  bool staged = false;
  auto clear_tail_slot = [&](uint32_t j0) {
    if (staged && (j0 & 1)) QG_HIP(hipMemsetAsync(a1, 0, SC_BACC_BYTES, ctx->stream));
  };
  Fr* loc = ctx->scratch_as<Fr>("sc_loc", NP);
  Fr* all = ctx->scratch_as<Fr>("sc_all", (size_t)world * NP);
  TablePtrs cur{};
  for (uint32_t i = 0; i < 8; i++) cur.src[i] = i < src.size() ? src[i] : nullptr;
  auto bufs = [&](Fr* base, size_t per) {
    TablePtrs t{};
    for (uint32_t i = 0; i < 8; i++) t.dst[i] = i < nslots ? base + per * i : nullptr;
    return t;
  };
  TablePtrs tX = bufs(X, NL / 2), tY = bufs(Y, std::max<size_t>(1, NL / 4));
  int fold = 0, parity = 0;
  {
    QgTimed tm(ctx, "sumcheck_round");
    for (uint32_t j = 0; j < js; j++) {
      const size_t npairs = (NL >> j) / 2;
      TablePtrs tp = cur;
      if (fold) {
        const TablePtrs& d = parity ? tY : tX;
        for (int i = 0; i < 8; i++) tp.dst[i] = d.dst[i];
      }
      int skip0 = launch_big<K, NP>(ctx, src, X, Y, NL, j, d_sp, h, npairs, ro, 0, loc, a0, a1, bar8);
      if (skip0 < 0) {
        skip0 = 0;
        staged = true;
        hipLaunchKernelGGL((k_sc_round<K, NP>), dim3(sc_round_blocks(ctx, npairs)), dim3(SC_BLOCK),
                           0, ctx->stream, tp, d_sp, h, npairs, fold, ro, j, 0, partial, loc);
      }
      QG_LAUNCH_CHECK();
      comm_allgather_bytes(ctx, loc, all, sizeof(Fr) * NP);
      hipLaunchKernelGGL((k_sc_finish<NP>), dim3(1), dim3(SC_BLOCK), 0, ctx->stream, d_sp, h, all,
                         world, ro, j, skip0);
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
    // this rank's source tables of round js: S entries per slot
    const size_t S = js == 0 ? NL : NL >> (js - 1);
    const size_t GN = (size_t)world * S;  // global size = 2^(nvars - js + 1) (js >= 1)
    const uint32_t ns = std::max(nslots, 1u);
    Fr* pack = ctx->scratch_as<Fr>("scg_pack", ns * S);
    Fr* gat = ctx->scratch_as<Fr>("scg_all", (size_t)world * ns * S);
    Fr* G = ctx->scratch_as<Fr>("scg_src", ns * GN);
    for (uint32_t i = 0; i < nslots; i++)
      QG_HIP(hipMemcpyAsync(pack + (size_t)i * S, cur.src[i], S * sizeof(Fr),
                            hipMemcpyDeviceToDevice, ctx->stream));
    if (nslots) {
      comm_allgather_bytes(ctx, pack, gat, (size_t)nslots * S * sizeof(Fr));
      hipLaunchKernelGGL(k_sc_gather_tables, dim3(div_up((size_t)world * nslots * S, 256)),
                         dim3(256), 0, ctx->stream, gat, world, nslots, S, G);
      QG_LAUNCH_CHECK();
    }
    // ping-pong buffers of the persistent rounds (run_rounds' capacities):
    // js == 0: round 0 does not fold, a >= GN/2, b >= GN/4 alternate from round 1;
    // js >= 1: round js folds into a (>= GN/2), then b (>= GN/4), a, ...
    Fr* A = ctx->scratch_as<Fr>("scg_a", ns * std::max<size_t>(1, GN / 2));
    Fr* B = ctx->scratch_as<Fr>("scg_b", ns * std::max<size_t>(1, GN / 4));
    TablePtrs t0{}, bufA{}, bufB{};
    for (uint32_t i = 0; i < 8; i++) {
      const bool u = i < nslots;
      t0.src[i] = u ? G + (size_t)i * GN : nullptr;
      Fr* a = u ? A + (size_t)i * std::max<size_t>(1, GN / 2) : nullptr;
      Fr* b = u ? B + (size_t)i * std::max<size_t>(1, GN / 4) : nullptr;
      if (js == 0) {
        bufA.dst[i] = a;
        bufB.dst[i] = b;
      } else {
        t0.dst[i] = a;
        bufA.dst[i] = b;
        bufB.dst[i] = a;
      }
    }
    const size_t PB = tail_pb(h.nslots, NP);
    const size_t pairs0 = ((size_t)1 << nvars >> js) / 2;
    // co-residency of the grid barrier: with the in-process loopback every rank
    // shares one device, so each persistent grid takes a 1/world share of the CUs
    const size_t cus = comm_is_loopback(ctx) ? std::max<size_t>(1, ctx->num_cus() / world)
                                             : (size_t)ctx->num_cus();
    clear_tail_slot(js);
    if (!launch_slice_tail<K, NP>(ctx, cus, t0, d_sp, h, nvars, js, js >= 1 ? 1 : 0, 0, ro, bar,
                                  (js & 1) ? a1 : a0, d_final, d_eval)) {
      const unsigned grid = (unsigned)std::max<size_t>(
          1, std::min<size_t>(persist_grid_cap<K, NP>(ctx, cus), (pairs0 + PB - 1) / PB));
      Fr* ppart = ctx->scratch_as<Fr>("sc_ppartial", (size_t)2 * grid * NP);
      hipLaunchKernelGGL((k_sc_tail<K, NP>), dim3(grid), dim3(TAIL_BLOCK), 0, ctx->stream, t0,
                         bufA, bufB, d_sp, h, nvars, js, js >= 1 ? 1 : 0, 0, ro, ppart, bar,
                         d_final, d_eval);
      QG_LAUNCH_CHECK();
    }
  }
  return js;
}

template <int K, int NP>
static uint32_t run_rounds_any(qg_ctx* ctx, uint32_t nvars, const std::vector<const Fr*>& src,
                               const SopDev* d_sp, SopHdr h, RoundOut ro, uint32_t* bar,
                               Fr* d_final, Fr* d_eval) {
  if (ctx->sharded) return run_rounds_dist<K, NP>(ctx, nvars, src, d_sp, h, ro, bar, d_final, d_eval);
  return run_rounds<K, NP>(ctx, nvars, src, d_sp, h, ro, bar, d_final, d_eval);
}

// inverse Vandermonde on nodes 0..np-1 for any np <= GEN_NPMAX: V[t][u]
// (Montgomery) with coefficient t of the interpolant = sum_u V[t][u] ev[u]
static std::vector<Fr> vinv_general(uint32_t np) {
  std::vector<Fr> V((size_t)np * np, Fr::zero());
  for (uint32_t j = 0; j < np; j++) {
    std::vector<Fr> poly(1, Fr::one());
    Fr den = Fr::one();
    for (uint32_t m = 0; m < np; m++) {
      if (m == j) continue;
      std::vector<Fr> np2(poly.size() + 1, Fr::zero());
      const Fr negm = fneg(from_u64<FrP>(m));
      for (size_t k = 0; k < poly.size(); k++) {
        np2[k] = np2[k] + poly[k] * negm;
        np2[k + 1] = np2[k + 1] + poly[k];
      }
      poly = np2;
      den = den * ((j >= m) ? from_u64<FrP>(j - m) : fneg(from_u64<FrP>(m - j)));
    }
    const Fr dinv = finv(den);
    for (uint32_t i = 0; i < np; i++) V[(size_t)i * np + j] = poly[i] * dinv;
  }
  return V;
}

// value of the postfix program on host values (Montgomery), per input table
static Fr host_eval_postfix(const qg_expr_op* prog, size_t len, const uint64_t* consts,
                            const std::vector<Fr>& in) {
  std::vector<Fr> st;
  for (size_t i = 0; i < len; i++) {
    const uint32_t op = prog[i].op, arg = prog[i].arg;
    if (op == QG_OP_INPUT) {
      st.push_back(in[arg]);
    } else if (op == QG_OP_CONST) {
      st.push_back(fr_import(consts + 4 * (size_t)arg));
    } else {
      const Fr b = st.back();
      st.pop_back();
      const Fr a = st.back();
      st.pop_back();
      st.push_back(op == QG_OP_ADD ? a + b : a * b);
    }
  }
  return st.back();
}

template <int NPP>
static void gen_round_kernels(qg_ctx* ctx, const Fr* const* d_ptrs, size_t half, uint32_t np,
                              const GenOp* d_ops, uint32_t len, const L9* d_c29, const L9* d_t29,
                              Fr* partial, Fr* d_out) {
  constexpr size_t PB = 256 / NPP;
  const unsigned grid = (unsigned)std::max<size_t>(1, std::min<size_t>(div_up(half, PB), 1024));
  hipLaunchKernelGGL((k_gen_eval<NPP>), dim3(grid), dim3(256), 0, ctx->stream, d_ptrs, half, np,
                     d_ops, len, d_c29, d_t29, partial);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL((k_gen_rows<NPP>), dim3(1), dim3(256), 0, ctx->stream, partial, grid, np,
                     d_out);
  QG_LAUNCH_CHECK();
}

// postfix program for the interpreter: used tables (first appearance), remapped
// ops, constants x 2^261; validates the program like expr_degree does
struct GenProg {
  std::vector<GenOp> ops;
  std::vector<uint32_t> used;
  std::vector<L9> c29;
};

static GenProg gen_prepare(const qg_expr_op* prog, size_t prog_len, const uint64_t* consts,
                           size_t nconsts, uint32_t ntables) {
  GenProg g;
  std::vector<uint32_t> slot_of(ntables, ~0u);
  g.ops.resize(prog_len);
  int depth = 0, maxd = 0;
  for (size_t i = 0; i < prog_len; i++) {
    const uint32_t op = prog[i].op, arg = prog[i].arg;
    if (op == QG_OP_INPUT) {
      QG_CHECK(arg < ntables, QG_ERR_INVALID, "expression input index out of range");
      if (slot_of[arg] == ~0u) {
        slot_of[arg] = (uint32_t)g.used.size();
        g.used.push_back(arg);
      }
      g.ops[i] = {op, slot_of[arg]};
      depth++;
    } else if (op == QG_OP_CONST) {
      QG_CHECK(arg < nconsts, QG_ERR_INVALID, "expression constant index out of range");
      g.ops[i] = {op, arg};
      depth++;
    } else {
      QG_CHECK(op == QG_OP_ADD || op == QG_OP_MUL, QG_ERR_INVALID, "unknown expression opcode");
      QG_CHECK(depth >= 2, QG_ERR_INVALID, "malformed expression (stack underflow)");
      g.ops[i] = {op, 0};
      depth--;
    }
    maxd = std::max(maxd, depth);
  }
  QG_CHECK(depth == 1, QG_ERR_INVALID, "malformed expression (stack size != 1)");
  QG_CHECK(maxd <= GEN_STACK, QG_ERR_UNSUPPORTED, "expression stack deeper than 32");
  g.c29.resize(std::max<size_t>(nconsts, 1));
  for (size_t i = 0; i < nconsts; i++)
    g.c29[i] = l9_of(plain_mul(from_mont(fr_import(consts + 4 * i)), pow2_mod_plain<FrP>(261)));
  return g;
}

// uploads ops and constants into scratch `tag`; returns (ops, consts) device pointers
static std::pair<GenOp*, L9*> gen_upload(qg_ctx* ctx, const GenProg& g, const std::string& tag) {
  const size_t ob = sizeof(GenOp) * std::max<size_t>(g.ops.size(), 1);
  const size_t ob_al = (ob + 63) & ~size_t(63);
  uint8_t* d = ctx->scratch_as<uint8_t>(tag, ob_al + sizeof(L9) * g.c29.size());
  QG_HIP(hipMemcpyAsync(d, g.ops.data(), sizeof(GenOp) * g.ops.size(), hipMemcpyHostToDevice,
                        ctx->stream));
  QG_HIP(hipMemcpyAsync(d + ob_al, g.c29.data(), sizeof(L9) * g.c29.size(), hipMemcpyHostToDevice,
                        ctx->stream));
  return {reinterpret_cast<GenOp*>(d), reinterpret_cast<L9*>(d + ob_al)};
}

// h(x) for the n rows of `tabs` into d_out (Logup / constraint-check fallback
// for expressions outside their compiled envelopes).  Synchronous: the host
// copies of the program are stack-local.
void expr_table_device(qg_ctx* ctx, size_t n, uint32_t ntables, const std::vector<const Fr*>& tabs,
                       const qg_expr_op* prog, size_t prog_len, const uint64_t* consts,
                       size_t nconsts, Fr* d_out) {
  const GenProg g = gen_prepare(prog, prog_len, consts, nconsts, ntables);
  auto dp = gen_upload(ctx, g, "gen_tab_prog");
  std::vector<const Fr*> hp(std::max<size_t>(g.used.size(), 1), nullptr);
  for (size_t s2 = 0; s2 < g.used.size(); s2++) hp[s2] = tabs[g.used[s2]];
  const Fr** d_ptrs = ctx->scratch_as<const Fr*>("gen_tab_ptrs", hp.size());
  QG_HIP(hipMemcpyAsync(d_ptrs, hp.data(), sizeof(Fr*) * hp.size(), hipMemcpyHostToDevice,
                        ctx->stream));
  hipLaunchKernelGGL(k_gen_table, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_ptrs, n,
                     dp.first, (uint32_t)g.ops.size(), dp.second, d_out);
  QG_LAUNCH_CHECK();
  ctx->sync();
}

// Sumcheck over the generic interpreter (see k_gen_eval); same transcript,
// proof and claim as the fast path (sumcheck.rs:28-114).  With a communicator
// attached (world W = 2^lw) each rank holds the 2^(nvars - lw) block of every
// table whose high index bits are its rank — the compiled path's decomposition:
// rounds j < m = nvars - lw pair local entries only, each rank's np round sums
// are allgathered and summed, and every rank runs the identical host transcript
// step; then every rank folds its block by r_{m-1} to one value per slot,
// allgathers those W x K values (the rank is the high index bits) and runs the
// last lw rounds redundantly on the gathered W-entry tables.
// cb != nullptr (qg_sumcheck_prove_cb): the caller's transcript absorbs each
// message and draws each challenge through the callback; `state` and
// `claimed_sum` are unused (the caller absorbed num_vars and the claim)
struct ScChallengeCb {
  qg_challenge_fn fn;
  void* user;
};

static void sumcheck_run_generic(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                                 const std::vector<const Fr*>& d_tables, const qg_expr_op* prog,
                                 size_t prog_len, const uint64_t* consts, size_t nconsts,
                                 const uint64_t claimed_sum[4], uint8_t state[32],
                                 uint64_t* round_coeffs, uint32_t* round_lens, uint64_t* point,
                                 uint64_t evaluation[4], const ScChallengeCb* cb = nullptr) {
  const uint32_t world = (uint32_t)ctx->world;
  uint32_t lw = 0;
  while ((1u << lw) < world) lw++;
  QG_CHECK((1u << lw) == world, QG_ERR_INVALID, "sharded sumcheck needs a power-of-two world");
  QG_CHECK(nvars >= lw, QG_ERR_INVALID, "sharded sumcheck needs nvars >= log2(world)");
  const uint32_t m = nvars - lw;  // rounds over local pairs
  const uint32_t width = expr_degree(prog, prog_len) + 1;
  const uint32_t np = width;
  QG_CHECK(np <= (uint32_t)GEN_NPMAX, QG_ERR_UNSUPPORTED, "expression degree above 31");
  const GenProg g = gen_prepare(prog, prog_len, consts, nconsts, ntables);
  const std::vector<uint32_t>& used = g.used;
  const uint32_t K = (uint32_t)used.size();
  const size_t NL = (size_t)1 << m;  // this rank's entries per table
  // t x 2^261 (plain integers, 29-bit limbs)
  std::vector<L9> t29(GEN_NPMAX);
  for (uint32_t t = 0; t < (uint32_t)GEN_NPMAX; t++)
    t29[t] = l9_of(plain_mul(from_u64_plain(t), pow2_mod_plain<FrP>(261)));
  const std::vector<Fr> V = vinv_general(np);
  const auto dprog = gen_upload(ctx, g, "gen_prog");
  const GenOp* d_ops = dprog.first;
  const L9* d_c29 = dprog.second;
  L9* d_t29 = ctx->scratch_as<L9>("gen_t29", GEN_NPMAX);
  QG_HIP(hipMemcpyAsync(d_t29, t29.data(), sizeof(L9) * GEN_NPMAX, hipMemcpyHostToDevice,
                        ctx->stream));
  const size_t Ks = std::max<uint32_t>(K, 1);
  // fold ping-pong (X: NL/2 per slot, Y: NL/4 per slot), gathered tables G
  // (W per slot) and their fold ping-pong (GX, GY: W/2, W/4 per slot)
  Fr* X = ctx->scratch_as<Fr>("gen_x", std::max<size_t>(1, (NL / 2) * Ks));
  Fr* Y = ctx->scratch_as<Fr>("gen_y", std::max<size_t>(1, (NL / 4) * Ks));
  Fr* G = ctx->scratch_as<Fr>("gen_g", (size_t)world * Ks);
  Fr* GX = ctx->scratch_as<Fr>("gen_gx", std::max<size_t>(1, (world / 2) * Ks));
  Fr* GY = ctx->scratch_as<Fr>("gen_gy", std::max<size_t>(1, (world / 4) * Ks));
  Fr* one = ctx->scratch_as<Fr>("gen_one", Ks);  // each slot folded to one value (gather send)
  // pointer arrays of the fold (src | dst) and of the evaluation, each its own
  // pinned staging slot: both are enqueued within one round, before its sync
  const Fr** d_ptrs_f = ctx->scratch_as<const Fr*>("gen_ptrs_f", 2 * Ks);
  const Fr** d_ptrs_e = ctx->scratch_as<const Fr*>("gen_ptrs_e", Ks);
  ScState* d_st = ctx->scratch_as<ScState>("gen_st", 1);
  Fr* partial = ctx->scratch_as<Fr>("gen_partial", (size_t)1024 * GEN_NPMAX);
  Fr* d_out = ctx->scratch_as<Fr>("gen_out", GEN_NPMAX);
  Fr* d_all = ctx->scratch_as<Fr>("gen_all", (size_t)world * std::max<size_t>(GEN_NPMAX, Ks));
  // transcript: append num_vars (usize) and claimed_sum (sumcheck.rs:35-36)
  if (!cb) {
    uint8_t b8[8], b32[32];
    u64_to_bytes(nvars, b8);
    transcript_append(state, b8, 8);
    fr_to_bytes(fr_import(claimed_sum), b32);
    transcript_append(state, b32, 32);
  }
  uint32_t npp = 4;
  while (npp < np) npp <<= 1;
  // per-slot table pointers of the current round's source
  std::vector<const Fr*> cur(Ks, nullptr);
  for (uint32_t s2 = 0; s2 < K; s2++) cur[s2] = d_tables[used[s2]];
  size_t cur_n = NL;  // entries per table of the current source
  auto upload_ptrs = [&](const Fr** d, const char* slot, const std::vector<const Fr*>& a,
                         const std::vector<Fr*>* b) {
    const size_t n = b ? 2 * Ks : Ks;
    const Fr** hp = reinterpret_cast<const Fr**>(ctx->pinned_get(slot, sizeof(Fr*) * n));
    for (size_t k = 0; k < Ks; k++) {
      hp[k] = a[k];
      if (b) hp[Ks + k] = (*b)[k];
    }
    QG_HIP(hipMemcpyAsync(d, hp, sizeof(Fr*) * n, hipMemcpyHostToDevice, ctx->stream));
  };
  // fold cur (cur_n entries per slot) by the challenge in d_st into dst[] (cur_n / 2 each)
  auto fold_into = [&](const std::vector<Fr*>& dst) {
    const size_t nq = cur_n / 2;
    if (K > 0) {
      upload_ptrs(d_ptrs_f, "gen_ptrs_f", cur, &dst);
      hipLaunchKernelGGL(k_gen_fold, dim3(div_up(nq * K, 256)), dim3(256), 0, ctx->stream,
                         d_ptrs_f, (Fr* const*)(d_ptrs_f + Ks), K, nq, d_st);
      QG_LAUNCH_CHECK();
      for (uint32_t s2 = 0; s2 < K; s2++) cur[s2] = dst[s2];
    }
    cur_n = nq;
  };
  std::vector<Fr> ev(np);
  Fr r = Fr::zero();
  bool pend_fold = false;  // the source still has to be folded by r
  int par = 0;             // next fold destination in the current phase: 0 -> X/GX, 1 -> Y/GY
  QgTimed tm(ctx, "sumcheck_round");
  for (uint32_t j = 0; j < nvars; j++) {
    if (j == m && lw > 0) {
      // gather: every slot folded to one value, allgathered; G[s][rank] = value
      if (pend_fold) {
        std::vector<Fr*> dst(Ks);
        for (uint32_t s2 = 0; s2 < K; s2++) dst[s2] = one + s2;
        fold_into(dst);
      } else {
        for (uint32_t s2 = 0; s2 < K; s2++)
          QG_HIP(hipMemcpyAsync(one + s2, cur[s2], sizeof(Fr), hipMemcpyDeviceToDevice, ctx->stream));
      }
      std::vector<Fr> all((size_t)world * Ks);
      if (K) {
        comm_allgather_bytes(ctx, one, d_all, sizeof(Fr) * K);
        QG_HIP(hipMemcpyAsync(all.data(), d_all, sizeof(Fr) * K * world, hipMemcpyDeviceToHost,
                              ctx->stream));
        ctx->sync();
        std::vector<Fr> gt((size_t)world * K);
        for (uint32_t rk = 0; rk < world; rk++)
          for (uint32_t s2 = 0; s2 < K; s2++) gt[(size_t)s2 * world + rk] = all[(size_t)rk * K + s2];
        QG_HIP(hipMemcpyAsync(G, gt.data(), sizeof(Fr) * gt.size(), hipMemcpyHostToDevice,
                              ctx->stream));
        ctx->sync();
      }
      for (uint32_t s2 = 0; s2 < K; s2++) cur[s2] = G + (size_t)world * s2;
      cur_n = world;
      pend_fold = false;
      par = 0;
    } else if (pend_fold) {
      std::vector<Fr*> dst(Ks);
      const bool gathered = j > m;  // rounds after the gather run on G
      Fr* base = gathered ? (par ? GY : GX) : (par ? Y : X);
      const size_t per = std::max<size_t>(1, gathered ? (par ? world / 4 : world / 2)
                                                       : (par ? NL / 4 : NL / 2));
      for (uint32_t s2 = 0; s2 < K; s2++) dst[s2] = base + per * s2;
      fold_into(dst);
      par ^= 1;
      pend_fold = false;
    }
    const size_t half = cur_n / 2;
    upload_ptrs(d_ptrs_e, "gen_ptrs_e", cur, nullptr);
    switch (npp) {
      case 4: gen_round_kernels<4>(ctx, d_ptrs_e, half, np, d_ops, (uint32_t)prog_len, d_c29, d_t29, partial, d_out); break;
      case 8: gen_round_kernels<8>(ctx, d_ptrs_e, half, np, d_ops, (uint32_t)prog_len, d_c29, d_t29, partial, d_out); break;
      case 16: gen_round_kernels<16>(ctx, d_ptrs_e, half, np, d_ops, (uint32_t)prog_len, d_c29, d_t29, partial, d_out); break;
      default: gen_round_kernels<32>(ctx, d_ptrs_e, half, np, d_ops, (uint32_t)prog_len, d_c29, d_t29, partial, d_out); break;
    }
    if (j < m && lw > 0) {
      // this rank's sums of the local pairs -> the global round sums
      comm_allgather_bytes(ctx, d_out, d_all, sizeof(Fr) * np);
      std::vector<Fr> all((size_t)world * np);
      QG_HIP(hipMemcpyAsync(all.data(), d_all, sizeof(Fr) * np * world, hipMemcpyDeviceToHost,
                            ctx->stream));
      ctx->sync();
      for (uint32_t t = 0; t < np; t++) {
        Fr a = Fr::zero();
        for (uint32_t rk = 0; rk < world; rk++) a = a + all[(size_t)rk * np + t];
        ev[t] = a;
      }
    } else {
      QG_HIP(hipMemcpyAsync(ev.data(), d_out, sizeof(Fr) * np, hipMemcpyDeviceToHost, ctx->stream));
      ctx->sync();
    }
    // coefficients, trim, absorb (u64 length + canonical coefficients), draw r
    std::vector<Fr> co(np);
    uint32_t len = 0;
    for (uint32_t t = 0; t < np; t++) {
      Fr a = Fr::zero();
      for (uint32_t u = 0; u < np; u++) a = a + V[(size_t)t * np + u] * ev[u];
      co[t] = a;
      if (!a.is_zero()) len = t + 1;
    }
    if (cb) {  // the caller's transcript: absorb the message, draw r_j
      std::vector<uint64_t> cm(4 * (size_t)std::max<uint32_t>(len, 1), 0);
      for (uint32_t t = 0; t < len; t++) fr_export(co[t], cm.data() + 4 * t);
      uint64_t rr[4] = {0, 0, 0, 0};
      QG_CHECK(cb->fn(cb->user, cm.data(), len, rr) == 0, QG_ERR_INVALID,
               "sumcheck challenge callback failed");
      r = fr_import(rr);
      Fr rc = r;
      reduce_once<FrP>(rc.v);
      QG_CHECK(rc == r, QG_ERR_INVALID, "challenge callback returned a non-reduced Fr");
    } else {
      std::vector<uint8_t> msg(8 + 32 * (size_t)len);
      u64_to_bytes(len, msg.data());
      for (uint32_t t = 0; t < len; t++) fr_to_bytes(co[t], msg.data() + 8 + 32 * t);
      transcript_append(state, msg.data(), msg.size());
      r = transcript_draw_fr(state);
    }
    for (uint32_t t = 0; t < width; t++)
      fr_export(t < len ? co[t] : Fr::zero(), round_coeffs + 4 * ((size_t)j * width + t));
    round_lens[j] = len;
    fr_export(r, point + 4 * j);
    // r x 2^261 for the next fold
    ScState* hs = reinterpret_cast<ScState*>(ctx->pinned_get("gen_st", sizeof(ScState)));
    memset(hs, 0, sizeof(ScState));
    const L9 r29 = l9_of(plain_mul(from_mont(r), pow2_mod_plain<FrP>(261)));
    for (int k = 0; k < 9; k++) hs->r29[k] = r29.v[k];
    QG_HIP(hipMemcpyAsync(d_st, hs, sizeof(ScState), hipMemcpyHostToDevice, ctx->stream));
    pend_fold = true;
  }
  // final fold with r_{n-1} on the host and h at the point (sumcheck.rs:93-99);
  // the last round's source holds 2 entries per slot (identical on every rank)
  std::vector<Fr> fin(ntables, Fr::zero());
  for (uint32_t s2 = 0; s2 < K; s2++) {
    Fr ab[2];
    QG_HIP(hipMemcpyAsync(ab, cur[s2], sizeof ab, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    for (Fr& x : ab) reduce_once<FrP>(x.v), reduce_once<FrP>(x.v);
    fin[used[s2]] = ab[0] + r * (ab[1] - ab[0]);
  }
  fr_export(host_eval_postfix(prog, prog_len, consts, fin), evaluation);
}

static void sumcheck_run(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                         const std::vector<const Fr*>& d_tables, const qg_expr_op* prog,
                         size_t prog_len, const uint64_t* consts, size_t nconsts,
                         const uint64_t claimed_sum[4], uint8_t state[32], uint64_t* round_coeffs,
                         uint32_t* round_lens, uint64_t* point, uint64_t evaluation[4]) {
  QG_CHECK(nvars >= 1 && nvars <= 40, QG_ERR_INVALID, "nvars out of range");
  std::shared_ptr<const ScProgram> P;
  try {
    P = get_program(prog, prog_len, consts, nconsts, ntables);
  } catch (const Error& e) {
    if (e.code != QG_ERR_UNSUPPORTED) throw;
    // outside the compiled envelope: the interpreted generic path
    return sumcheck_run_generic(ctx, nvars, ntables, d_tables, prog, prog_len, consts, nconsts,
                                claimed_sum, state, round_coeffs, round_lens, point, evaluation);
  }
  const uint32_t width = P->width;

  // transcript: append num_vars (usize) and claimed_sum (sumcheck.rs:35-36)
  ScState hs;
  memset(&hs, 0, sizeof hs);
  {
    uint8_t st[32], b8[8], b32[32];
    memcpy(st, state, 32);
    u64_to_bytes(nvars, b8);
    transcript_append(st, b8, 8);
    fr_to_bytes(fr_import(claimed_sum), b32);
    transcript_append(st, b32, 32);
    memcpy(hs.state, st, 32);
  }

  // one device region: ScState | barrier counters | chal | coeffs | final (8 slots +
  // evaluation) | lens.  ScState and the counters are (re)initialised per call.
  const size_t o_bar = sizeof(ScState);
  const size_t o_chal = sumcheck_o_bacc0(nvars) + SC_BACC_BYTES;  // after the accumulator
  const size_t o_coeffs = o_chal + sizeof(Fr) * nvars;
  const size_t o_final = o_coeffs + sizeof(Fr) * (size_t)nvars * width;
  const size_t o_lens = o_final + sizeof(Fr) * 9;
  const size_t io_bytes = o_lens + sizeof(uint32_t) * nvars;
  uint8_t* io = ctx->scratch_as<uint8_t>("sc_io", io_bytes);
  SopDev* d_sp = ctx->scratch_as<SopDev>("sc_prog", 1);
  // the device copy holds program P->id while the slot's allocation generation
  // is unchanged (arena.h: never an address)
  const std::string memo =
      ctx->arena.derived_key(std::to_string(P->id), 1, ctx->scratch_gen("sc_prog"));
  if (!ctx->arena.check("sc_prog", memo)) {
    QG_HIP(hipMemcpyAsync(d_sp, &P->img, sizeof(SopDev), hipMemcpyHostToDevice, ctx->stream));
    ctx->arena.commit("sc_prog", memo);
  }
  uint8_t* hio = reinterpret_cast<uint8_t*>(ctx->pinned_get("sc_io", io_bytes));
  memset(hio, 0, o_chal);
  memcpy(hio, &hs, sizeof hs);
  QG_HIP(hipMemcpyAsync(io, hio, o_chal, hipMemcpyHostToDevice, ctx->stream));
  uint32_t* bar = reinterpret_cast<uint32_t*>(io + o_bar);

  std::vector<const Fr*> src;
  for (uint32_t u : P->used) src.push_back(d_tables[u]);
  RoundOut ro{reinterpret_cast<ScState*>(io), reinterpret_cast<Fr*>(io + o_chal),
              reinterpret_cast<Fr*>(io + o_coeffs), reinterpret_cast<uint32_t*>(io + o_lens),
              width};
  Fr* d_final = reinterpret_cast<Fr*>(io + o_final);
  Fr* d_eval = d_final + 8;
  const uint32_t np = P->hdr.np;
  const size_t nsrc = src.size();
  // (with no used slots, nslots = 0 and loads are skipped)
  uint32_t tail0;
  if (np <= 4) {
    if (nsrc <= 4) tail0 = run_rounds_any<4, 4>(ctx, nvars, src, d_sp, P->hdr, ro, bar, d_final, d_eval);
    else tail0 = run_rounds_any<8, 4>(ctx, nvars, src, d_sp, P->hdr, ro, bar, d_final, d_eval);
  } else if (np <= 8) {
    if (nsrc <= 4) tail0 = run_rounds_any<4, 8>(ctx, nvars, src, d_sp, P->hdr, ro, bar, d_final, d_eval);
    else tail0 = run_rounds_any<8, 8>(ctx, nvars, src, d_sp, P->hdr, ro, bar, d_final, d_eval);
  } else {
    tail0 = run_rounds_any<8, 16>(ctx, nvars, src, d_sp, P->hdr, ro, bar, d_final, d_eval);
  }

  QG_HIP(hipMemcpyAsync(hio, io, io_bytes, hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  const std::vector<uint8_t> h(hio, hio + io_bytes);
  QG_CHECK(reinterpret_cast<const ScState*>(h.data())->err == 0, QG_ERR_DEVICE,
           "sumcheck: grid barrier timed out (persistent blocks not co-resident)");
  memcpy(state, h.data(), 32);
  memcpy(round_lens, h.data() + o_lens, sizeof(uint32_t) * nvars);
  const Fr* hc = reinterpret_cast<const Fr*>(h.data() + o_coeffs);
  // every round kernel writes canonical words (finish_core canon_out): the
  // Montgomery pass after the challenge stays off the device's critical path
  (void)tail0;
  for (size_t i = 0; i < (size_t)nvars * width; i++) fr_export(to_mont(hc[i]), round_coeffs + 4 * i);
  const Fr* hp = reinterpret_cast<const Fr*>(h.data() + o_chal);
  for (uint32_t i = 0; i < nvars; i++) fr_export(hp[i], point + 4 * i);
  fr_export(reinterpret_cast<const Fr*>(h.data() + o_final)[8], evaluation);
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
  if (ctx->sharded) {
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

#ifdef QG_SC_TRACE
int qg_debug_sc_trace(uint64_t* out, size_t n) {
  if (n > 2048 + 4 * 1536) n = 2048 + 4 * 1536;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sc_trace), n * 8) == hipSuccess ? QG_OK : QG_ERR_DEVICE;
}
int qg_debug_sc_wtrace(uint64_t* out, size_t n) {
  if (n > 4 * 512 * 8 * 2) n = 4 * 512 * 8 * 2;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sc_wtrace), n * 8) == hipSuccess ? QG_OK : QG_ERR_DEVICE;
}
#endif

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

int qg_eq_table_dev(qg_ctx* ctx, const uint64_t* point, size_t nvars, qg_buf* out) {
  if (!ctx || (!point && nvars) || !out || nvars > 40) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    // with a communicator: this rank's block (high index bits = rank)
    uint32_t lw = 0;
    while ((1 << lw) < ctx->world) lw++;
    QG_CHECK((1 << lw) == ctx->world, QG_ERR_INVALID, "world size must be a power of two");
    QG_CHECK(nvars >= lw, QG_ERR_INVALID, "nvars must be at least log2(world)");
    const uint32_t m = (uint32_t)nvars - lw;
    const size_t N = (size_t)1 << m;
    QG_CHECK(out->n >= N, QG_ERR_INVALID, "output buffer too short");
    Fr* d_z = ctx->scratch_as<Fr>("eq_z", nvars ? nvars : 1);
    fr_upload(ctx, d_z, point, nvars);
    eq_table_device(ctx, d_z, m, out->d);
    if (lw) {
      Fr f = Fr::one();
      for (uint32_t j = m; j < nvars; j++) {
        const Fr zj = fr_import(point + 4 * j);
        f = f * ((((uint32_t)ctx->rank >> (j - m)) & 1u) ? zj : Fr::one() - zj);
      }
      Fr* d_f = ctx->scratch_as<Fr>("eq_f", 1);
      QG_HIP(hipMemcpyAsync(d_f, &f, sizeof(Fr), hipMemcpyHostToDevice, ctx->stream));
      hipLaunchKernelGGL(k_scale, dim3(div_up(N, 256)), dim3(256), 0, ctx->stream, out->d, N, d_f);
      QG_LAUNCH_CHECK();
    }
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

int qg_sumcheck_prove_cb(qg_ctx* ctx, uint32_t nvars, uint32_t ntables,
                         const qg_buf* const* tables, const qg_expr_op* prog, size_t prog_len,
                         const uint64_t* consts, size_t nconsts, qg_challenge_fn challenge,
                         void* user, uint64_t* round_coeffs, uint32_t* round_lens,
                         uint64_t* point, uint64_t evaluation[4]) {
  if (!ctx || (!tables && ntables) || !prog || !challenge || !round_coeffs || !round_lens ||
      !point || !evaluation || (!consts && nconsts))
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
    const ScChallengeCb cb{challenge, user};
    const uint64_t zero[4] = {0, 0, 0, 0};
    uint8_t unused[32] = {0};
    sumcheck_run_generic(ctx, nvars, ntables, d, prog, prog_len, consts, nconsts, zero, unused,
                         round_coeffs, round_lens, point, evaluation, &cb);
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
