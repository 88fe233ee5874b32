// Multilinear PCS opening passes for gfx950 — replaces
//   KZG::open                          pcs/src/kzg.rs:75-96
//   MLEvalProof::compute_pr / prove    pcs/src/mlpcs.rs:52-124
//   InnerProductProof::compute_s_polynomial  pcs/src/ipa.rs:122-157
//
//  * compute_pr == the eq table (identity pinned by the KATs at
//    mlpcs.rs:226-242): built in O(2^n) on the device, no IFFT.
//  * y = p(x) and q = (p - y)/(X - x) come out of ONE suffix-Horner scan
//    s_i = c_i + x s_{i+1}:  y = s_0, q_i = s_{i+1}.  The scan is blocked:
//    per-chunk zero-carry values, a recursive scan of the chunk carries with
//    multiplier x^B, then a per-chunk apply pass.
//  * S_k = sum_i (f_{i+k+1} g_i + g_{i+k+1} f_i) is the upper half of
//    h = f*rev(g) + rev(f)*g.  Two forward NTTs (F, G) suffice:
//    NTT(rev f)[j] = w^{j(M-1)} F[-j], so H[j] = w^{j(M-1)} (F[j]G[-j] + F[-j]G[j]).
//  * Every commitment is the device MSM (msm.hip) over device-resident data.
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "blake3.h"
#include "common.h"
#include "field29.h"

using namespace qg;

namespace qg {

static constexpr int ML_BLOCK = 256;
static constexpr int SH_B = 32;  // suffix-Horner chunk length

// ---------------------------------------------------------------- reductions
QG_DEV Fr shfl_xor_fr2(const Fr& a, int m) {
  Fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = __shfl_xor(a.v[i], m, 64);
  return r;
}

QG_DEV Fr block_sum_fr(Fr v, Fr* lds) {
  for (int m = 32; m > 0; m >>= 1) v = v + shfl_xor_fr2(v, m);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  Fr acc = Fr::zero();
  if (threadIdx.x == 0)
    for (int w = 0; w < nw; w++) acc = acc + lds[w];
  __syncthreads();
  return acc;
}

__global__ void __launch_bounds__(ML_BLOCK)
    k_dot(const Fr* __restrict__ f, const Fr* __restrict__ g, size_t n, Fr* __restrict__ partial) {
  __shared__ Fr lds[ML_BLOCK / 64];
  Fr acc = Fr::zero();
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    acc = acc + f[i] * g[i];
  acc = block_sum_fr(acc, lds);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__global__ void __launch_bounds__(ML_BLOCK)
    k_sum(const Fr* __restrict__ in, size_t n, Fr* __restrict__ out) {
  __shared__ Fr lds[ML_BLOCK / 64];
  Fr acc = Fr::zero();
  for (size_t i = threadIdx.x; i < n; i += blockDim.x) acc = acc + in[i];
  acc = block_sum_fr(acc, lds);
  if (threadIdx.x == 0) *out = acc;
}

// <f, g> into device memory (no host round trip)
static void dot_to_device(qg_ctx* ctx, const Fr* f, const Fr* g, size_t n, Fr* d_out) {
  if (n == 0) {
    QG_HIP(hipMemsetAsync(d_out, 0, sizeof(Fr), ctx->stream));
    return;
  }
  QgTimed tm(ctx, "inner_product");
  unsigned blocks = (unsigned)std::min<size_t>(2048, div_up(n, ML_BLOCK));
  Fr* part = ctx->scratch_as<Fr>("dot_part", blocks);
  hipLaunchKernelGGL(k_dot, dim3(blocks), dim3(ML_BLOCK), 0, ctx->stream, f, g, n, part);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sum, dim3(1), dim3(ML_BLOCK), 0, ctx->stream, part, (size_t)blocks, d_out);
  QG_LAUNCH_CHECK();
}

static Fr dot_device(qg_ctx* ctx, const Fr* f, const Fr* g, size_t n) {
  if (n == 0) return Fr::zero();
  QgTimed tm(ctx, "inner_product");
  unsigned blocks = (unsigned)std::min<size_t>(2048, div_up(n, ML_BLOCK));
  Fr* part = ctx->scratch_as<Fr>("dot_part", blocks + 1);
  hipLaunchKernelGGL(k_dot, dim3(blocks), dim3(ML_BLOCK), 0, ctx->stream, f, g, n, part);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sum, dim3(1), dim3(ML_BLOCK), 0, ctx->stream, part, (size_t)blocks,
                     part + blocks);
  QG_LAUNCH_CHECK();
  Fr r;
  QG_HIP(hipMemcpyAsync(&r, part + blocks, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  return r;
}

// ---------------------------------------------------------------- suffix Horner
// A_k = sum_{i in chunk k} c_i x^(i - start_k)
__global__ void k_sh_local(const Fr* __restrict__ c, size_t L, Fr x, Fr* __restrict__ A) {
  size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t s = k * SH_B;
  if (s >= L) return;
  size_t e = s + SH_B < L ? s + SH_B : L;
  Fr acc = Fr::zero();
  for (size_t i = e; i-- > s;) acc = c[i] + x * acc;
  A[k] = acc;
}

// s_i for every i given T_{k+1} (suffix value at the start of chunk k+1)
__global__ void k_sh_apply(const Fr* __restrict__ c, size_t L, Fr x, const Fr* __restrict__ T,
                           size_t nchunks, Fr* __restrict__ s_out) {
  size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t s = k * SH_B;
  if (s >= L) return;
  size_t e = s + SH_B < L ? s + SH_B : L;
  Fr acc = (k + 1 < nchunks) ? T[k + 1] : Fr::zero();
  for (size_t i = e; i-- > s;) {
    acc = c[i] + x * acc;
    s_out[i] = acc;
  }
}

// small case: one thread
__global__ void k_sh_serial(const Fr* __restrict__ c, size_t L, Fr x, Fr* __restrict__ s_out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  Fr acc = Fr::zero();
  for (size_t i = L; i-- > 0;) {
    acc = c[i] + x * acc;
    s_out[i] = acc;
  }
}

// s = suffix Horner of c (length L) at x: s_i = c_i + x s_{i+1}
static void suffix_horner(qg_ctx* ctx, const Fr* c, size_t L, const Fr& x, Fr* s, int depth = 0) {
  if (L == 0) return;
  if (L <= SH_B) {
    hipLaunchKernelGGL(k_sh_serial, dim3(1), dim3(64), 0, ctx->stream, c, L, x, s);
    QG_LAUNCH_CHECK();
    return;
  }
  const size_t nch = (L + SH_B - 1) / SH_B;
  Fr* A = ctx->scratch_as<Fr>("sh_A" + std::to_string(depth), nch);
  Fr* T = ctx->scratch_as<Fr>("sh_T" + std::to_string(depth), nch);
  hipLaunchKernelGGL(k_sh_local, dim3(div_up(nch, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream, c,
                     L, x, A);
  QG_LAUNCH_CHECK();
  // T_k = A_k + x^B T_{k+1}
  Fr xb = fpow_small(x, SH_B);
  suffix_horner(ctx, A, nch, xb, T, depth + 1);
  hipLaunchKernelGGL(k_sh_apply, dim3(div_up(nch, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream, c, L,
                     x, T, nch, s);
  QG_LAUNCH_CHECK();
}

// Batched form (up to 4 independent scans per launch, blockIdx.y = scan) in
// 9 x 29-bit limbs (each step c_i + x s_{i+1}: a canonical coefficient plus a
// product < 2p, so one conditional subtraction keeps s < 2p): the per-chunk Horner chain is the latency of the whole
// recursion, and the 29-bit multiply's dependent latency is half the 32-bit
// one's.  x is passed as x 2^261 (plain limbs), so mul29 keeps the arkworks
// scale of the coefficients.
struct ShJob {
  const Fr* c;  // coefficients (arkworks form)
  size_t L;
  L9 x;         // x 2^261 mod p
  Fr* A;        // chunk values (local pass)
  const Fr* T;  // chunk carries (apply pass)
  size_t nch;
  Fr* s;        // output suffixes
};
struct ShJobs {
  ShJob j[4];
};

// The apply pass on a full chunk runs software-pipelined: its coefficients
// come in groups of SH_G, the next group's loads issued before the current
// group's dependent products and stores (one load round trip per group instead
// of per step, which the stores would otherwise pin in program order); a short
// last chunk loops.  Every suffix value is written.
static constexpr int SH_G = 4;
__device__ __forceinline__ void sh_apply_chunk(const Fr* __restrict__ c, Fr* __restrict__ out,
                                               size_t s, size_t e, const F29<FrP>& x,
                                               F29<FrP> acc) {
  if (e - s == SH_B) {
    Fr cur[SH_G], nxt[SH_G];
#pragma unroll
    for (int j = 0; j < SH_G; j++) cur[j] = c[s + SH_B - SH_G + j];
#pragma unroll
    for (int g = SH_B / SH_G - 1; g >= 0; g--) {
      if (g > 0) {
#pragma unroll
        for (int j = 0; j < SH_G; j++) nxt[j] = c[s + (size_t)(g - 1) * SH_G + j];
      }
      // keeps the scheduler from hoisting later groups' loads above this
      // group's products
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = SH_G - 1; j >= 0; j--) {
        acc = red2p29(add29(to29(cur[j]), mul29(x, acc)));
        out[s + (size_t)g * SH_G + j] = from29(canon29(acc));
      }
      if (g > 0) {
#pragma unroll
        for (int j = 0; j < SH_G; j++) cur[j] = nxt[j];
      }
    }
  } else {
    for (size_t i = e; i-- > s;) {
      acc = red2p29(add29(to29(c[i]), mul29(x, acc)));
      out[i] = from29(canon29(acc));
    }
  }
}

__global__ void k_sh_local_b(ShJobs jb) {
  const ShJob& J = jb.j[blockIdx.y];
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t s = k * SH_B;
  if (s >= J.L) return;
  const size_t e = s + SH_B < J.L ? s + SH_B : J.L;
  const F29<FrP> x = F29<FrP>::from_l9(J.x);
  F29<FrP> acc = F29<FrP>::zero();
  // no stores in this chain: an unrolled loop lets the loads run ahead
#pragma unroll 4
  for (size_t i = e; i-- > s;) acc = red2p29(add29(to29(J.c[i]), mul29(x, acc)));
  J.A[k] = from29(canon29(acc));
}

__global__ void k_sh_apply_b(ShJobs jb) {
  const ShJob& J = jb.j[blockIdx.y];
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t s = k * SH_B;
  if (s >= J.L) return;
  const size_t e = s + SH_B < J.L ? s + SH_B : J.L;
  const F29<FrP> x = F29<FrP>::from_l9(J.x);
  const F29<FrP> acc0 = (k + 1 < J.nch) ? to29(J.T[k + 1]) : F29<FrP>::zero();
  sh_apply_chunk(J.c, J.s, s, e, x, acc0);
}

__global__ void k_sh_serial_b(ShJobs jb) {
  const ShJob& J = jb.j[blockIdx.y];
  if (threadIdx.x != 0) return;
  const F29<FrP> x = F29<FrP>::from_l9(J.x);
  F29<FrP> acc = F29<FrP>::zero();
  for (size_t i = J.L; i-- > 0;) {
    acc = red2p29(add29(to29(J.c[i]), mul29(x, acc)));
    J.s[i] = from29(canon29(acc));
  }
}

struct ShIn {
  const Fr* c;
  size_t L;
  Fr x;  // Montgomery
  Fr* s;
};

static L9 x261_of(const Fr& x) {
  const Fr t = from_mont(to_mont(from_mont(x)) * to_mont(pow2_mod_plain<FrP>(261)));
  const F29<FrP> r = to29(t);
  L9 o{};
  for (int i = 0; i < 9; i++) o.v[i] = r.l[i];
  return o;
}

// s_i = c_i + x s_{i+1} for up to 4 independent (c, L, x) at once
static void suffix_horner_batch(qg_ctx* ctx, const std::vector<ShIn>& in, int depth = 0) {
  std::vector<ShIn> small, big;
  for (const ShIn& q : in)
    if (q.L > SH_B) big.push_back(q);
    else if (q.L > 0) small.push_back(q);
  QG_CHECK(in.size() <= 4, QG_ERR_ASSERT, "suffix-Horner batch of at most 4");
  if (!small.empty()) {
    ShJobs jb{};
    for (size_t q = 0; q < small.size(); q++)
      jb.j[q] = {small[q].c, small[q].L, x261_of(small[q].x), nullptr, nullptr, 0, small[q].s};
    hipLaunchKernelGGL(k_sh_serial_b, dim3(1, (unsigned)small.size()), dim3(64), 0, ctx->stream, jb);
    QG_LAUNCH_CHECK();
  }
  if (big.empty()) return;
  ShJobs jb{};
  std::vector<ShIn> up;
  size_t maxch = 0;
  for (size_t q = 0; q < big.size(); q++) {
    const size_t nch = (big[q].L + SH_B - 1) / SH_B;
    const std::string tag = std::to_string(depth) + "_" + std::to_string(q);
    Fr* A = ctx->scratch_as<Fr>("shb_A" + tag, nch);
    Fr* T = ctx->scratch_as<Fr>("shb_T" + tag, nch);
    jb.j[q] = {big[q].c, big[q].L, x261_of(big[q].x), A, T, nch, big[q].s};
    up.push_back({A, nch, fpow_small(big[q].x, SH_B), T});  // T_k = A_k + x^B T_{k+1}
    maxch = std::max(maxch, nch);
  }
  const dim3 grid((unsigned)div_up(maxch, ML_BLOCK), (unsigned)big.size());
  hipLaunchKernelGGL(k_sh_local_b, grid, dim3(ML_BLOCK), 0, ctx->stream, jb);
  QG_LAUNCH_CHECK();
  suffix_horner_batch(ctx, up, depth + 1);
  hipLaunchKernelGGL(k_sh_apply_b, grid, dim3(ML_BLOCK), 0, ctx->stream, jb);
  QG_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- NTT
// Radix-2 NTT passes of up to 10 stages each on LDS tiles of 1024 elements
// held as 9 x 29-bit limbs (SoA: conflict-free), so a 2^24-point transform is
// three HBM round trips instead of one per stage.  A pass over stages
// [s0, s0 + B) works on tiles of 2^B "mid" indices x L consecutive "lo"
// indices (L = 1024 / 2^B): element (mid, l) is index
//   hi 2^(s0+B) + mid 2^s0 + lo0 + l,
// so every global access is a run of L consecutive Fr (L >= 8 above the first
// pass).  36 KB tiles let four blocks share a CU (16 waves; the 2048-element
// 72 KB tiles fit two: S polynomial at 2^23 -5 %, profiles/r04_ntt_tile_ab.txt).  Forward: DIF (natural in, bit-reversed out); inverse: DIT
// (bit-reversed in, natural out) -- no bit-reversal pass at all.  Data stay in
// arkworks form (x 2^256): twiddles are stored as w^k 2^261, so mul29 keeps the
// scale.  Every value is < 2p inside a pass, canonical (< p) when stored.
#ifndef QG_NTT_LGT
#define QG_NTT_LGT 10
#endif
static constexpr int NTT_LGT = QG_NTT_LGT;
static constexpr int NTT_T = 1 << NTT_LGT;  // elements per tile
#ifndef QG_NTT_THREADS
#define QG_NTT_THREADS 256
#endif
static constexpr int NTT_THREADS = QG_NTT_THREADS;
using R29 = F29<FrP>;

struct NttPass {
  int s0, B, lgL;
};

// stage ranges: [0, min(10, logn)) first (contiguous tiles), then chunks of at
// most 7 stages (runs of >= 8 elements)
static std::vector<NttPass> ntt_plan(int logn) {
  std::vector<NttPass> v;
  int s = 0;
  while (s < logn) {
    const int B = std::min(s == 0 ? NTT_LGT : 7, logn - s);
    int lgL = std::min(NTT_LGT - B, s);  // L <= 2^s0 (lo range)
    lgL = std::min(lgL, logn - B);       // tile <= n
    v.push_back({s, B, lgL});
    s += B;
  }
  return v;
}

QG_DEV R29 lds_get29(const uint32_t* sh, int e) {
  R29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = sh[i * NTT_T + e];
  return r;
}
QG_DEV void lds_put29(uint32_t* sh, int e, const R29& v) {
#pragma unroll
  for (int i = 0; i < 9; i++) sh[i * NTT_T + e] = v.l[i];
}

// Twiddles by stage ("pyramid"): stage s's butterflies use w^(j 2^(logn-1-s))
// for j < 2^s, stored contiguously at pyr[2^s - 1 + j] (2^logn - 1 entries,
// twice the flat table).  Neighbouring butterflies of a stage have
// neighbouring j, so a wave's twiddle loads are runs of consecutive 32-B
// entries instead of one cache line per lane (the flat table's stride is
// 2^(logn-1-s) entries).  Built once per (table, logn) from the flat powers.
__global__ void k_tw_pyramid(const Fr* __restrict__ flat, int logn, Fr* __restrict__ pyr) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)1 << logn;
  if (i + 1 >= n) return;
  const int st = 63 - __clzll((unsigned long long)(i + 1));  // stage of entry i
  const size_t j = i + 1 - ((size_t)1 << st);
  pyr[i] = flat[j << (logn - 1 - st)];
}

// DIF (forward) or DIT (inverse) stages [s0, s0+B) on every tile.
//   in:  n entries (entries >= nin read as zero)
//   out: n entries, or only indices [win_lo, win_hi) written to out - win_lo
//   tw:  w^k 2^261 (Fr words) as the stage pyramid (pyr != 0) or flat, k < n/2
template <bool DIF>
__global__ void __launch_bounds__(NTT_THREADS)
    k_ntt_pass(const Fr* __restrict__ in, size_t nin, Fr* __restrict__ out,
               const Fr* __restrict__ tw, int pyr, int logn, int s0, int B, int lgL,
               size_t win_lo, size_t win_hi) {
  __shared__ uint32_t sh[9 * NTT_T];
  const int lgT = B + lgL, T = 1 << lgT;
  const int L = 1 << lgL;
  const size_t tid = threadIdx.x;
  // tile id -> (hi, lo group)
  const size_t ngroups = ((size_t)1 << s0) >> lgL;
  const size_t hi = blockIdx.x / ngroups, lo0 = (blockIdx.x % ngroups) << lgL;
  const size_t base = (hi << (s0 + B)) + lo0;
  for (int e = (int)tid; e < T; e += NTT_THREADS) {
    const size_t i = base + ((size_t)(e >> lgL) << s0) + (e & (L - 1));
    R29 v = R29::zero();
    if (i < nin) v = to29(in[i]);
    lds_put29(sh, e, v);
  }
  __syncthreads();
  for (int k = 0; k < B; k++) {
    const int b = DIF ? B - 1 - k : k;  // mid bit of this stage
    const int s = s0 + b;
    // butterflies p and p + NTT_THREADS together: their two Montgomery products
    // run as interleaved chains (mul29t2); a lone last one alone
    for (int p0 = (int)tid; p0 < T / 2; p0 += 2 * NTT_THREADS) {
      const bool two = p0 + NTT_THREADS < T / 2;
      int e0[2], e1[2];
      R29 u[2], v[2], w[2];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int p = h && two ? p0 + NTT_THREADS : p0;
        const int l = p & (L - 1), q = p >> lgL;
        const int mid0 = ((q >> b) << (b + 1)) | (q & ((1 << b) - 1));
        e0[h] = (mid0 << lgL) | l;
        e1[h] = e0[h] | (1 << (b + lgL));
        const size_t j = ((size_t)(mid0 & ((1 << b) - 1)) << s0) + lo0 + l;  // i0 mod 2^s
        w[h] = to29(tw[pyr ? ((size_t)1 << s) - 1 + j : j << (logn - 1 - s)]);
        u[h] = lds_get29(sh, e0[h]);
        v[h] = lds_get29(sh, e1[h]);
      }
      R29 t[2];
      if (DIF) {
        mul29t2(sub29(u[0], v[0]), w[0], sub29(u[1], v[1]), w[1], t[0], t[1]);
      } else {
        mul29t2(v[0], w[0], v[1], w[1], t[0], t[1]);
      }
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (h && !two) break;
        if (DIF) {
          lds_put29(sh, e0[h], red2p29(add29(u[h], v[h])));
          lds_put29(sh, e1[h], t[h]);
        } else {
          lds_put29(sh, e0[h], red2p29(add29(u[h], t[h])));
          // u + 2p - t in [0, 4p) (u, t < 2p): one conditional subtraction
          lds_put29(sh, e1[h], red2p29(subk29(u[h], t[h], F29P<FrP>::K2)));
        }
      }
    }
    __syncthreads();
  }
  for (int e = (int)tid; e < T; e += NTT_THREADS) {
    const size_t i = base + ((size_t)(e >> lgL) << s0) + (e & (L - 1));
    if (i >= win_lo && i < win_hi) out[i - win_lo] = from29(canon29(lds_get29(sh, e)));
  }
}

// the stage pyramid of the flat twiddle table in scratch slot `src` (one
// derived slot per source slot; valid for the source's current build stamp and
// its own allocation generation, never for an address)
static const Fr* ntt_pyramid(qg_ctx* ctx, const Fr* flat, const std::string& src, int logn) {
  const std::string tag = "ntt_pyr:" + src;
  const size_t n = (size_t)1 << logn;
  Fr* pyr = ctx->scratch_as<Fr>(tag, std::max<size_t>(1, n - 1));
  const uint64_t st = ctx->arena.stamp(src);
  const std::string key = ctx->arena.derived_key(std::to_string(logn), st, ctx->scratch_gen(tag));
  if (!ctx->arena.check(tag, key, st)) {
    hipLaunchKernelGGL(k_tw_pyramid, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, flat, logn,
                       pyr);
    QG_LAUNCH_CHECK();
    ctx->arena.commit(tag, key);
  }
  return pyr;
}

// runs every pass in place on `a` (the first pass reads `in`), direction by DIF
static void ntt_run(qg_ctx* ctx, bool dif, const Fr* in, size_t nin, Fr* a, const Fr* tw,
                    const std::string& tw_slot, int logn, size_t win_lo, size_t win_hi,
                    Fr* win_out) {
  // QG_NTT_FLAT=1: twiddles from the flat table (A/B runs)
  static const bool flat = [] {
    const char* e = getenv("QG_NTT_FLAT");
    return e && atoi(e) != 0;
  }();
  const Fr* pyr = flat ? tw : ntt_pyramid(ctx, tw, tw_slot, logn);
  const int pmode = flat ? 0 : 1;
  std::vector<NttPass> plan = ntt_plan(logn);
  if (dif) std::reverse(plan.begin(), plan.end());
  const size_t n = (size_t)1 << logn;
  for (size_t k = 0; k < plan.size(); k++) {
    const NttPass& P = plan[k];
    const bool last = k + 1 == plan.size();
    const Fr* src = k == 0 ? in : a;
    const size_t ns = k == 0 ? nin : n;
    Fr* dst = last && win_out ? win_out : a;
    const size_t lo = last && win_out ? win_lo : 0, hi = last && win_out ? win_hi : n;
    const unsigned blocks = (unsigned)(n >> (P.B + P.lgL));
    if (dif)
      hipLaunchKernelGGL(k_ntt_pass<true>, dim3(blocks), dim3(NTT_THREADS), 0, ctx->stream, src, ns,
                         dst, pyr, pmode, logn, P.s0, P.B, P.lgL, lo, hi);
    else
      hipLaunchKernelGGL(k_ntt_pass<false>, dim3(blocks), dim3(NTT_THREADS), 0, ctx->stream, src,
                         ns, dst, pyr, pmode, logn, P.s0, P.B, P.lgL, lo, hi);
    QG_LAUNCH_CHECK();
  }
}

// x 2^256 (arkworks) -> x 2^261 in place: mul29 by 2^266
__global__ void k_fr_to261(Fr* __restrict__ a, size_t n, L9 c) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) a[i] = from29(canon29(mul29(to29(a[i]), R29::from_l9(c))));
}

// twM in the combine's order: out[k] = in[bitrev(k)] c 2^-261 (the table is
// built once per (logn, M); read in natural order by k_s_combine_br, its
// loads are coalesced instead of one line per lane)
__global__ void k_fr_to261_br(const Fr* __restrict__ in, int logn, L9 c, Fr* __restrict__ out) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= ((size_t)1 << logn)) return;
  const size_t j = (size_t)(__brevll((unsigned long long)k) >> (64 - logn));
  out[k] = from29(canon29(mul29(to29(in[j]), R29::from_l9(c))));
}

// bit-reversed domain: H_br[k] = tw_k (F[j] G[-j] + F[-j] G[j]), j = bitrev(k);
// bitrev(-j) = k with every bit below k's top set bit flipped.  twMb[k] =
// twM[bitrev(k)] carries w^{j(M-1)} n^-1 2^266, so mul29 of the 2^251-scaled
// products lands in arkworks form with 1/n folded in.
__global__ void k_s_combine_br(const Fr* __restrict__ F, const Fr* __restrict__ G,
                               const Fr* __restrict__ twMb, int logn, Fr* __restrict__ H) {
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t n = (size_t)1 << logn;
  if (k >= n) return;
  size_t kn = 0;
  if (k) {
    const int hb = 63 - __clzll((unsigned long long)k);
    kn = k ^ (((size_t)1 << hb) - 1);
  }
  const R29 a = to29(F[k]), bb = to29(G[kn]), c = to29(F[kn]), d = to29(G[k]);
  const R29 v = red2p29(add29(mul29(a, bb), mul29(c, d)));
  H[k] = from29(canon29(mul29(v, to29(twMb[k]))));
}

// ---- the inverse transform at half size (round 6) ------------------------
// With P_j = F_j G_{-j} + F_{-j} G_j (P_{-j} = P_j) the S polynomial is
// S_k = p_{k+1} (k < M - 1) for p = IDFT_n(P): H_j = w^{j(M-1)} P_j / n only
// shifts p by M - 1, and p is even (p_{-d} = p_d).  Split p by parity
// (N2 = n / 2, w2 = w^2):
//   p_{2e}     = a_e / n,  a = IDFT_N2(A),  A_j = P_j + P_{j+N2}
//   p_{2e+1}   = b_e / n,  b = IDFT_N2(B),  B_j = (P_j - P_{j+N2}) w^{-j}
// A is even (A_{N2-j} = A_j), so a is even; B_{N2-j} = w2^j B_j, so
// b_{-e} = b_{e-1}.  One half-size inverse of D = A + B gives d = a + b, and
// d_e - d_{-e} = (a_e + b_e) - (a_e + b_{e-1}) = b_e - b_{e-1}: b is b_0 plus
// a prefix sum of d_e - d_{N2-e}, with b_0 = sum_j B_j, and a = d - b.  So the
// size-n inverse NTT becomes a size-n/2 one plus O(n) combine / scan passes.
// In the bit-reversed domain P_j and P_{j+N2} sit at 2t and 2t + 1
// (t = bitrev_{N2}(j)), and D_j is needed at position t of the half-size
// DIT's bit-reversed input: each thread makes one D from two adjacent P.
// twD[t] = w^{-bitrev(t)} n^-1 2^266, c1 = n^-1 2^266: mul29 of the 2^251-scaled
// values lands in arkworks form with 1/n folded in (as twM does).
// bpart[block] = the block's sum of B_j / n (for b_0).
__global__ void __launch_bounds__(256)
    k_s_combine_half(const Fr* __restrict__ F, const Fr* __restrict__ G, const Fr* __restrict__ twD,
                     L9 c1, int logn, Fr* __restrict__ D, Fr* __restrict__ bpart) {
  __shared__ Fr red[256];
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t N2 = (size_t)1 << (logn - 1);
  Fr bn = Fr::zero();
  if (t < N2) {
    R29 P[2];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const size_t q = 2 * t + h;
      size_t kn = 0;
      if (q) {
        const int hb = 63 - __clzll((unsigned long long)q);
        kn = q ^ (((size_t)1 << hb) - 1);
      }
      const R29 a = to29(F[q]), bb = to29(G[kn]), c = to29(F[kn]), d = to29(G[q]);
      P[h] = red2p29(add29(mul29(a, bb), mul29(c, d)));  // < 2p, x 2^251
    }
    const R29 A = add29(P[0], P[1]);                                      // < 4p, lazy
    const R29 B = normfull29(subk29(P[0], P[1], F29P<FrP>::K2));          // < 4p, normalized
    const R29 An = mul29(A, R29::from_l9(c1));
    const R29 Bn = mul29(B, to29(twD[t]));
    D[t] = from29(canon29(red2p29(add29(An, Bn))));
    bn = from29(canon29(Bn));
  }
  red[threadIdx.x] = bn;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) bpart[blockIdx.x] = red[0];
}

// out[0] = sum of in[0 .. n) (one block)
__global__ void __launch_bounds__(1024) k_fr_sum(const Fr* __restrict__ in, size_t n, Fr* __restrict__ out) {
  __shared__ Fr red[1024];
  Fr acc = Fr::zero();
  for (size_t i = threadIdx.x; i < n; i += 1024) acc = acc + in[i];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 512; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] = red[threadIdx.x] + red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

// b_e = b_0 + sum_{t=1..e} (d_t - d_{N2-t}), e = 0 .. E: tiles of SYM_TILE
// entries, a local inclusive prefix per tile (Q) and the tile totals (tot)
static constexpr int SYM_PER = 8;
static constexpr int SYM_TILE = 256 * SYM_PER;
__global__ void __launch_bounds__(256)
    k_sym_tiles(const Fr* __restrict__ d, size_t N2, size_t E, Fr* __restrict__ Q, Fr* __restrict__ tot) {
  __shared__ Fr sh[256];
  const size_t e0 = (size_t)blockIdx.x * SYM_TILE + (size_t)threadIdx.x * SYM_PER;
  Fr v[SYM_PER];
  Fr run = Fr::zero();
#pragma unroll
  for (int k = 0; k < SYM_PER; k++) {
    const size_t e = e0 + k;
    Fr dl = Fr::zero();
    if (e >= 1 && e <= E) dl = d[e] - d[N2 - e];
    run = run + dl;
    v[k] = run;
  }
  sh[threadIdx.x] = run;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // Hillis-Steele inclusive scan of the thread totals
    const Fr add = (int)threadIdx.x >= o ? sh[threadIdx.x - o] : Fr::zero();
    __syncthreads();
    sh[threadIdx.x] = sh[threadIdx.x] + add;
    __syncthreads();
  }
  const Fr before = threadIdx.x ? sh[threadIdx.x - 1] : Fr::zero();
#pragma unroll
  for (int k = 0; k < SYM_PER; k++)
    if (e0 + k <= E) Q[e0 + k] = before + v[k];
  if (threadIdx.x == 255) tot[blockIdx.x] = sh[255];
}

// tot[i] <- b_0 + sum_{i' < i} tot[i'] (one block)
__global__ void __launch_bounds__(1024) k_sym_top(Fr* __restrict__ tot, int ntiles, const Fr* __restrict__ b0) {
  __shared__ Fr sh[1024];
  const int per = (ntiles + 1023) / 1024;
  const int base = threadIdx.x * per;
  Fr sum = Fr::zero();
  for (int k = 0; k < per; k++)
    if (base + k < ntiles) sum = sum + tot[base + k];
  sh[threadIdx.x] = sum;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const Fr add = (int)threadIdx.x >= o ? sh[threadIdx.x - o] : Fr::zero();
    __syncthreads();
    sh[threadIdx.x] = sh[threadIdx.x] + add;
    __syncthreads();
  }
  Fr run = b0[0] + (threadIdx.x ? sh[threadIdx.x - 1] : Fr::zero());
  for (int k = 0; k < per; k++)
    if (base + k < ntiles) {
      const Fr t = tot[base + k];
      tot[base + k] = run;
      run = run + t;
    }
}

// S_{2e-1} = p_{2e} = d_e - b_e (e >= 1), S_{2e} = p_{2e+1} = b_e, for the
// k = 2e - 1, 2e below M - 1
__global__ void k_sym_out(const Fr* __restrict__ d, const Fr* __restrict__ Q, const Fr* __restrict__ tot,
                          size_t M, size_t E, Fr* __restrict__ S) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e > E) return;
  const Fr b = tot[e / SYM_TILE] + Q[e];
  if (2 * e + 2 <= M) S[2 * e] = b;                   // k = 2e <= M - 2
  if (e >= 1 && 2 * e + 1 <= M) S[2 * e - 1] = d[e] - b;  // k = 2e - 1 <= M - 2
}

__global__ void k_powers_ml(Fr base, size_t n, int K, Fr* out) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t i0 = t * (size_t)K;
  if (i0 >= n) return;
  Fr x = fpow_small(base, (uint64_t)i0);
  for (int j = 0; j < K && i0 + j < n; j++) {
    out[i0 + j] = x;
    x = x * base;
  }
}

// host-side 256-bit exponent power
static Fr fr_pow_big(Fr a, const uint32_t e[8]) {
  Fr r = Fr::one();
  for (int i = 7; i >= 0; i--)
    for (int b = 31; b >= 0; b--) {
      r = fsqr(r);
      if ((e[i] >> b) & 1u) r = r * a;
    }
  return r;
}

// primitive 2^logn-th root of unity: 5^((r-1)/2^logn)
static Fr root_of_unity(int logn) {
  uint32_t e[8];
  for (int i = 0; i < 8; i++) e[i] = FrP::P[i];
  e[0] -= 1;  // r - 1 (low limb of r is odd)
  for (int k = 0; k < logn; k++) {  // shift right by logn
    for (int i = 0; i < 8; i++) e[i] = (e[i] >> 1) | (i < 7 ? (e[i + 1] << 31) : 0u);
  }
  return fr_pow_big(from_u64<FrP>(5), e);
}

// plain-integer product x y mod r (host)
static Fr ml_plain_mul(const Fr& x, const Fr& y) { return from_mont(to_mont(x) * to_mont(y)); }

// twiddle tables w^k 2^261 (k < n/2) for w = root_of_unity(logn) and its
// inverse in scratch slots `tag` and `tag`+"i", cached per transform size and
// allocation generation; every build stamps both slots, which invalidates the
// tables derived from them (ntt_pyramid, ntt_tw_bitrev)
static void ntt_twiddles(qg_ctx* ctx, int logn, Fr** tw, Fr** twi,
                         const std::string& tag = "ntt_tw") {
  const size_t n = (size_t)1 << logn, h = std::max<size_t>(n / 2, 1);
  *tw = ctx->scratch_as<Fr>(tag, h);
  *twi = ctx->scratch_as<Fr>(tag + "i", h);
  const std::string key = std::to_string(logn) + "|g" + std::to_string(ctx->scratch_gen(tag)) +
                          "," + std::to_string(ctx->scratch_gen(tag + "i"));
  if (ctx->arena.check(tag, key)) return;
  const Fr w = root_of_unity(logn), wi = finv(w);
  const int K = 64;
  const L9 c = F29P<FrP>::TO261;
  hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(h, K), 256)), dim3(256), 0, ctx->stream, w, h,
                     K, *tw);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(h, K), 256)), dim3(256), 0, ctx->stream, wi,
                     h, K, *twi);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_fr_to261, dim3(div_up(h, 256)), dim3(256), 0, ctx->stream, *tw, h, c);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_fr_to261, dim3(div_up(h, 256)), dim3(256), 0, ctx->stream, *twi, h, c);
  QG_LAUNCH_CHECK();
  ctx->arena.bump(tag);
  ctx->arena.bump(tag + "i");
  ctx->arena.commit(tag, key);
}

// Transform of the eq table without an NTT.  g = eq(., z) over nz variables is
// the coefficient vector of G(X) = prod_t ((1 - z_t) + z_t X^(2^t)), so
//   G(w^j) = Q_0(j),  Q_t(j) = ((1 - z_t) + z_t w^(j 2^t)) Q_{t+1}(j),  Q_nz = 1,
// where Q_t depends only on j mod 2^(L-t).  In the bit-reversed order of the
// DIF outputs (k' = bitrev_{L-t}(j mod 2^(L-t))) the recursion is streaming:
//   Q_t[k'] = f_t(k') Q_{t+1}[k' >> 1].
// One level per launch, 2^(L-t) entries; ~2 multiplies per entry over all
// levels (~4 x 2^L in total) instead of L/2 per entry of a forward NTT.
// Q is kept in arkworks form (x 2^256), the factor in the 2^261 domain.
// With twb = the flat table in bit-reversed order (twb[i] = tw[bitrev_{L-1}(i)]),
// level t's twiddle w^(bitrev_{L-t}(k) 2^t) is twb[k >> 1], negated for odd k
// (the top bit of the exponent is k's low bit, w^(2^(L-1)) = -1): consecutive
// entries read consecutive table words instead of one cache line per lane.
__global__ void k_eqdft_level(const Fr* __restrict__ qnext, L9 a261, L9 z261,
                              const Fr* __restrict__ twb, int logn, int t, Fr* __restrict__ q) {
  const size_t len = (size_t)1 << (logn - t);
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= len) return;
  R29 w = to29(twb[k >> 1]);
  if (k & 1) w = sub29(R29::zero(), w);  // lazy 4p - w
  // a261 < p (host-canonical), the product < 2p: one conditional subtraction
  const R29 f = red2p29(add29(R29::from_l9(a261), mul29(R29::from_l9(z261), w)));
  const R29 qn = qnext ? to29(qnext[k >> 1]) : to29(Fr::one());
  q[k] = from29(canon29(mul29(f, qn)));
}

// The small top levels of the same recursion in ONE launch (they were ~5 us
// launches of a few thousand entries each): level tmin's entry k is
//   Q_tmin[k] = prod_{t = tmin}^{nz-1} f_t(k >> (t - tmin)),
// every factor from the same bit-reversed table (twb[k' >> 1], negated for odd
// k'), two factors per step as interleaved products.  A thread per entry of
// level tmin (2^(logn - tmin) <= EQ_TOP_LEN entries).
static constexpr int EQ_TOP_MAXL = 32;
static constexpr int EQ_TOP_LOG = 16;  // levels of <= 2^16 entries are fused
struct EqTopConsts {
  L9 a[EQ_TOP_MAXL], z[EQ_TOP_MAXL];  // level tmin + i: (1 - z_t), z_t in the 2^261 domain
};
__global__ void __launch_bounds__(256)
    k_eqdft_top(EqTopConsts cs, uint32_t nlev, const Fr* __restrict__ twb, int logn, int tmin,
                Fr* __restrict__ q) {
  const size_t len = (size_t)1 << (logn - tmin);
  const size_t k = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= len) return;
  R29 acc = to29(Fr::one());
  for (uint32_t i = 0; i < nlev; i++) {
    const size_t kk = k >> i;
    R29 w = to29(twb[kk >> 1]);
    if (kk & 1) w = sub29(R29::zero(), w);  // lazy 4p - w
    // a < p (host-canonical), the product < 2p: one conditional subtraction
    const R29 f = red2p29(add29(R29::from_l9(cs.a[i]), mul29(R29::from_l9(cs.z[i]), w)));
    acc = mul29(f, acc);  // arkworks form (x 2^256) kept: f carries 2^261
  }
  q[k] = from29(canon29(acc));
}

// twb[i] = tw[bitrev_{L-1}(i)] for i < 2^(L-1) (one entry for L <= 1)
__global__ void k_tw_bitrev(const Fr* __restrict__ tw, int logn, size_t h, Fr* __restrict__ twb) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= h) return;
  const size_t j = logn > 1 ? (size_t)(__brevll((unsigned long long)i) >> (65 - logn)) : 0;
  twb[i] = tw[j];
}

// the flat twiddle table of scratch slot `src` in bit-reversed order (keyed
// like ntt_pyramid)
static const Fr* ntt_tw_bitrev(qg_ctx* ctx, const Fr* tw, const std::string& src, int logn) {
  const std::string tag = "ntt_twb:" + src;
  const size_t h = logn > 1 ? (size_t)1 << (logn - 1) : 1;
  Fr* twb = ctx->scratch_as<Fr>(tag, h);
  const uint64_t st = ctx->arena.stamp(src);
  const std::string key = ctx->arena.derived_key(std::to_string(logn), st, ctx->scratch_gen(tag));
  if (!ctx->arena.check(tag, key, st)) {
    hipLaunchKernelGGL(k_tw_bitrev, dim3(div_up(h, 256)), dim3(256), 0, ctx->stream, tw, logn, h,
                       twb);
    QG_LAUNCH_CHECK();
    ctx->arena.commit(tag, key);
  }
  return twb;
}

static L9 l9_of29(const Fr& x) {
  const R29 t = to29(x);
  L9 c{};
  for (int i = 0; i < 9; i++) c.v[i] = t.l[i];
  return c;
}

// S polynomial (M - 1 coefficients, untrimmed) of f (nf) and g (ng), device in/out.
// eq_z (nz variables, host Montgomery): g is eq(., eq_z) over 2^nz entries, and
// its transform comes from the product formula (k_eqdft_level) instead of an NTT.
// f_id: the allocation id of the qg_buf behind f (qg_buf::alloc_id, never
// reused; 0 = unknown).  reuse_f: the caller guarantees f's contents are
// unchanged since the last call that transformed this same buffer; F is then
// reused when this context still holds that transform (arena memo "ntt_F_src":
// f's allocation id and offset, length, size, and the generation of F's slot).
static void s_poly_device(qg_ctx* ctx, const Fr* f, size_t nf, const Fr* g, size_t ng, Fr* S,
                          const uint64_t* eq_z = nullptr, size_t nz = 0, bool reuse_f = false,
                          uint64_t f_id = 0, size_t f_off = 0) {
  const size_t M = nf > ng ? nf : ng;
  if (M <= 1) return;
  QgTimed tm(ctx, "s_polynomial");
  int logn = 0;
  while (((size_t)1 << logn) < 2 * M - 1) logn++;
  QG_CHECK(logn <= 28, QG_ERR_UNSUPPORTED, "S-polynomial NTT beyond 2-adicity");
  if (logn < 1) logn = 1;
  const size_t n = (size_t)1 << logn;
  Fr* F = ctx->scratch_as<Fr>("ntt_F", n);
  Fr* G = ctx->scratch_as<Fr>("ntt_G", n);
  Fr* H = ctx->scratch_as<Fr>("ntt_H", n);
  // w^{j(M-1)} n^-1 2^266 for j < n: powers of w^{M-1} (x 2^256, staged in H),
  // then x n^-1 2^271 via mul29 into twM in bit-reversed order.  Depends on
  // (logn, M) only: cached per context in one of four slots by (logn, M), so a
  // prover alternating between a few opening sizes (HyperPlonk: the witness
  // and its public rows) does not rebuild it per opening.
  // QG_S_FULL_INVERSE=1: the size-n inverse (k_s_combine_br + DIT of H) instead
  // of the half-size one (A/B runs); read per call
  const char* fi = getenv("QG_S_FULL_INVERSE");
  const bool half_inverse = !(fi && atoi(fi) != 0);
  Fr *tw, *twi;
  ntt_twiddles(ctx, logn, &tw, &twi);
  Fr* twM = nullptr;
  Fr* twD = nullptr;
  if (half_inverse) {
    // w^{-j} n^-1 2^266 for j < n / 2 in bit-reversed order: depends on logn only
    twD = ctx->scratch_as<Fr>("ntt_twD", n / 2);
    const std::string memo = ctx->arena.derived_key(std::to_string(logn), 1, ctx->scratch_gen("ntt_twD"));
    if (!ctx->arena.check("ntt_twD", memo)) {
      const Fr wi = finv(root_of_unity(logn));
      const int K = 64;
      hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(n / 2, K), 256)), dim3(256), 0, ctx->stream,
                         wi, n / 2, K, H);
      QG_LAUNCH_CHECK();
      const Fr ninv_plain = from_mont(finv(from_u64<FrP>(n)));
      const L9 c9 = l9_of29(ml_plain_mul(ninv_plain, pow2_mod_plain<FrP>(271)));
      hipLaunchKernelGGL(k_fr_to261_br, dim3(div_up(n / 2, 256)), dim3(256), 0, ctx->stream, H,
                         logn - 1, c9, twD);
      QG_LAUNCH_CHECK();
      ctx->arena.commit("ntt_twD", memo);
    }
  }
  const std::string twm_key = std::to_string(logn) + ":" + std::to_string(M);
  bool twm_hit = false;  // the memo below decides; the LRU only picks the slot
  const std::string twm_slot =
      half_inverse ? std::string() : "ntt_twM#" + std::to_string(ctx->twm_lru.slot_for(twm_key, &twm_hit));
  if (!half_inverse) twM = ctx->scratch_as<Fr>(twm_slot, n);
  const std::string twm_memo =
      half_inverse ? std::string() : ctx->arena.derived_key(twm_key, 1, ctx->scratch_gen(twm_slot));
  if (!half_inverse && !ctx->arena.check(twm_slot, twm_memo)) {
    const Fr w = root_of_unity(logn);
    const Fr wM = fpow_small(w, (uint64_t)(M - 1));
    const int K = 64;
    hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(n, K), 256)), dim3(256), 0, ctx->stream, wM,
                       n, K, H);
    QG_LAUNCH_CHECK();
    const Fr ninv_plain = from_mont(finv(from_u64<FrP>(n)));
    const Fr cM = ml_plain_mul(ninv_plain, pow2_mod_plain<FrP>(271));
    L9 c9{};
    {
      const R29 t = to29(cM);
      for (int i = 0; i < 9; i++) c9.v[i] = t.l[i];
    }
    hipLaunchKernelGGL(k_fr_to261_br, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, H, logn, c9,
                       twM);
    QG_LAUNCH_CHECK();
    ctx->arena.commit(twm_slot, twm_memo);
  }
  // forward DIF of f and g (zero-extended), bit-reversed outputs
  const std::string fkey =
      f_id ? ctx->arena.derived_key(std::to_string(f_id) + "+" + std::to_string(f_off) + ":" +
                                        std::to_string(nf) + ":" + std::to_string(logn),
                                    ctx->arena.stamp("ntt_tw"), ctx->scratch_gen("ntt_F"))
           : std::string();
  if (!(reuse_f && f_id && ctx->arena.memo["ntt_F_src"] == fkey)) {
    ctx->arena.memo["ntt_F_src"].clear();
    ntt_run(ctx, true, f, nf, F, tw, "ntt_tw", logn, 0, 0, nullptr);
    ctx->arena.memo["ntt_F_src"] = fkey;
  }
  if (eq_z && nz >= 1 && ((size_t)1 << nz) == ng && (int)nz < logn) {
    // levels t = nz-1 .. 0 ping-pong between G and H (H is free until the combine),
    // ending in G (t = 0: 2^logn entries, bit-reversed order)
    const Fr* twb = ntt_tw_bitrev(ctx, tw, "ntt_tw", logn);
    // the levels of <= 2^EQ_TOP_LOG entries (t >= tmin) in one launch into the
    // array level tmin would have been written to, then one launch per level
    static const bool eq_top = [] {
      const char* e = getenv("QG_EQ_TOP");  // 0: one launch per level (A/B runs)
      return !(e && atoi(e) == 0);
    }();
    int t_hi = (int)nz - 1;  // highest level still to run per launch
    const int tmin = std::max(0, logn - EQ_TOP_LOG);
    if (eq_top && tmin < (int)nz && (int)nz - tmin <= EQ_TOP_MAXL) {
      EqTopConsts cs{};
      for (int t = tmin; t < (int)nz; t++) {
        const Fr z = fr_import(eq_z + 4 * t);
        const Fr zp = from_mont(z), ap = from_mont(Fr::one() - z);
        cs.z[t - tmin] = l9_of29(ml_plain_mul(zp, pow2_mod_plain<FrP>(261)));
        cs.a[t - tmin] = l9_of29(ml_plain_mul(ap, pow2_mod_plain<FrP>(261)));
      }
      Fr* dst = (tmin & 1) == 0 ? G : H;
      const size_t len = (size_t)1 << (logn - tmin);
      hipLaunchKernelGGL(k_eqdft_top, dim3(div_up(len, 256)), dim3(256), 0, ctx->stream, cs,
                         (uint32_t)(nz - tmin), twb, logn, tmin, dst);
      QG_LAUNCH_CHECK();
      t_hi = tmin - 1;
    }
    for (int t = t_hi; t >= 0; t--) {
      const Fr z = fr_import(eq_z + 4 * t);
      const Fr zp = from_mont(z), ap = from_mont(Fr::one() - z);
      const L9 z9 = l9_of29(ml_plain_mul(zp, pow2_mod_plain<FrP>(261)));
      const L9 a9 = l9_of29(ml_plain_mul(ap, pow2_mod_plain<FrP>(261)));
      Fr* dst = (t & 1) == 0 ? G : H;
      const Fr* src = t == (int)nz - 1 ? nullptr : ((t & 1) == 0 ? H : G);  // level t + 1
      const size_t len = (size_t)1 << (logn - t);
      hipLaunchKernelGGL(k_eqdft_level, dim3(div_up(len, 256)), dim3(256), 0, ctx->stream, src,
                         a9, z9, twb, logn, t, dst);
      QG_LAUNCH_CHECK();
    }
  } else {
    ntt_run(ctx, true, g, ng, G, tw, "ntt_tw", logn, 0, 0, nullptr);
  }
  if (!half_inverse) {
    hipLaunchKernelGGL(k_s_combine_br, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, F, G, twM,
                       logn, H);
    QG_LAUNCH_CHECK();
    // inverse DIT of H (bit-reversed in, natural out); the last pass writes only
    // h[M .. 2M-1) = S
    ntt_run(ctx, false, H, n, H, twi, "ntt_twi", logn, M, 2 * M - 1, S);
    return;
  }
  // the inverse at half size (k_s_combine_half): D into H's first half,
  // the half-size DIT in place, then b by a prefix scan into S
  const size_t N2 = n / 2;
  const unsigned cblocks = div_up(N2, 256);
  Fr* bpart = ctx->scratch_as<Fr>("s_bpart", (size_t)cblocks + 1);
  const Fr ninv_plain = from_mont(finv(from_u64<FrP>(n)));
  const L9 c1 = l9_of29(ml_plain_mul(ninv_plain, pow2_mod_plain<FrP>(266)));
  hipLaunchKernelGGL(k_s_combine_half, dim3(cblocks), dim3(256), 0, ctx->stream, F, G, twD, c1, logn,
                     H, bpart);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_fr_sum, dim3(1), dim3(1024), 0, ctx->stream, bpart, (size_t)cblocks,
                     bpart + cblocks);
  QG_LAUNCH_CHECK();
  Fr *twh, *twhi;
  ntt_twiddles(ctx, logn - 1, &twh, &twhi, "ntt_twh");
  ntt_run(ctx, false, H, N2, H, twhi, "ntt_twhi", logn - 1, 0, 0, nullptr);
  const size_t E = (M - 1) / 2;  // b_e, a_e for e <= E cover S_0 .. S_{M-2}
  const size_t ntiles = E / SYM_TILE + 1;
  QG_CHECK(ntiles <= 1024 * 64, QG_ERR_UNSUPPORTED, "S-polynomial scan too large");
  Fr* tot = ctx->scratch_as<Fr>("s_symtot", ntiles);
  hipLaunchKernelGGL(k_sym_tiles, dim3((unsigned)ntiles), dim3(256), 0, ctx->stream, H, N2, E, G, tot);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sym_top, dim3(1), dim3(1024), 0, ctx->stream, tot, (int)ntiles,
                     bpart + cblocks);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sym_out, dim3(div_up(E + 1, 256)), dim3(256), 0, ctx->stream, H, G, tot, M, E,
                     S);
  QG_LAUNCH_CHECK();
}

// highest nonzero index + 1: per-thread max over a grid-stride range of
// [lo, hi), wave max by shuffles, one atomic per wave (a contended atomic per
// element cost 0.75 ms at 2^22) into *out.  The tail launch (the last 16K
// entries) also stamps *tail with (call generation << 40 | its max); the body
// launch skips a block when *tail holds this call's generation and a nonzero
// max: the tail covered the higher indices, so any body index is below the
// answer (a full body scan at 2^23 is 110 us; most vectors end in a nonzero
// value).
//
// Round 6: the skip used to read *out itself, which the body launch's own
// blocks write: a block that started after another block of the same launch
// had posted its maximum exited without scanning its range, so the length
// came out short (81152 or 81664 instead of 81920 for HyperPlonk's trimmed
// full witness at 2^14 rows, whose tail is zero) whenever the launch's blocks
// did not all start before the first one finished - timing-dependent, seen
// with the MSM batches' side streams active (micro/handover_dbg.py,
// profiles/r06_handover_diagnosis.txt).  A short length gives a wrong
// quotient, so a wrong KZG opening proof; no opening proof enters the
// transcript, so only a verifier or a proof-by-proof comparison sees it.
__global__ void __launch_bounds__(256)
    k_last_nonzero(const Fr* __restrict__ a, size_t lo, size_t hi, unsigned long long* tail,
                   uint64_t gen, int body, unsigned long long* out) {
  if (body) {
    const unsigned long long t = __hip_atomic_load(tail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((t >> 40) == gen && (t & ((1ull << 40) - 1)) != 0) return;
  }
  unsigned long long m = 0;
  for (size_t i = lo + (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi;
       i += (size_t)gridDim.x * blockDim.x)
    if (!a[i].is_zero()) m = i + 1;
  for (int k = 32; k > 0; k >>= 1) {
    const unsigned long long o = __shfl_xor(m, k, 64);
    m = o > m ? o : m;
  }
  if ((threadIdx.x & 63) == 0) {
    if (m) atomicMax(out, m);
    if (!body) atomicMax(tail, (gen << 40) | m);  // this call's stamp, even when m = 0
  }
}

// trimmed length of a device vector: the last 16K entries first (8 blocks),
// then the rest, skipped when the tail held a nonzero
static void trim_launch(qg_ctx* ctx, const Fr* a, size_t n, unsigned long long* d) {
  QG_HIP(hipMemsetAsync(d, 0, sizeof(unsigned long long), ctx->stream));
  if (n == 0) return;
  constexpr size_t TAIL = 16384;
  const size_t body = n > TAIL ? n - TAIL : 0;
  // one stamp word per context, reused in stream order; generations only grow,
  // so a stamp of an earlier call never matches (a wrapped counter only costs
  // the skip)
  unsigned long long* tail = ctx->scratch_as<unsigned long long>("trim_tail", 1);
  const uint64_t gen = (++ctx->trim_gen) & 0xffffffull;
  hipLaunchKernelGGL(k_last_nonzero, dim3((unsigned)std::min<size_t>(8, div_up(n - body, 256))),
                     dim3(256), 0, ctx->stream, a, body, n, tail, gen, 0, d);
  QG_LAUNCH_CHECK();
  if (body) {
    const unsigned blocks = (unsigned)std::min<size_t>(2048, div_up(body, 256));
    hipLaunchKernelGGL(k_last_nonzero, dim3(blocks), dim3(256), 0, ctx->stream, a, (size_t)0,
                       body, tail, gen, 1, d);
    QG_LAUNCH_CHECK();
  }
}

static size_t trimmed_len(qg_ctx* ctx, const Fr* a, size_t n) {
  if (n == 0) return 0;
  unsigned long long* d = ctx->scratch_as<unsigned long long>("trim_len", 1);
  trim_launch(ctx, a, n, d);
  unsigned long long h = 0;
  QG_HIP(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  return (size_t)h;
}

// four KZG::open quotients at once (the ML opening's poly and S at r and
// 1/r) on their trimmed lengths `Lt` (the caller's), one batched
// suffix-Horner recursion, and the four values y = s_0 queued into pinned
// memory (h_y[4]) without a round trip: the caller reads them after its next
// synchronization (the quotient MSMs')
// `slot` keeps the quotient buffers of several openings apart (a batch of
// openings commits all of its quotients at once, mle_open_batch_device).
static void kzg_quotients_batch(qg_ctx* ctx, const qg_srs* srs, const Fr* const polys[4],
                                const size_t Lt[4], const Fr xs[4], qg_kzg_opening* const outs[4],
                                std::vector<const Fr*>& qs, std::vector<size_t>& qns, Fr* h_y,
                                size_t slot = 0) {
  std::vector<ShIn> jobs;
  Fr* s[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int i = 0; i < 4; i++) {
    fr_export(xs[i], outs[i]->x);
    if (Lt[i] == 0) continue;
    QG_CHECK(Lt[i] - 1 <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
    s[i] = ctx->scratch_as<Fr>("open_s#" + std::to_string(4 * slot + i), Lt[i]);
    jobs.push_back({polys[i], Lt[i], xs[i], s[i]});
  }
  {
    QgTimed tm(ctx, "kzg_division");
    suffix_horner_batch(ctx, jobs);
  }
  Fr* d_y = ctx->scratch_as<Fr>("open_y#" + std::to_string(slot), 4);
  QG_HIP(hipMemsetAsync(d_y, 0, 4 * sizeof(Fr), ctx->stream));
  for (int i = 0; i < 4; i++)
    if (s[i])
      QG_HIP(hipMemcpyAsync(d_y + i, s[i], sizeof(Fr), hipMemcpyDeviceToDevice, ctx->stream));
  QG_HIP(hipMemcpyAsync(h_y, d_y, 4 * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  qs.clear();
  qns.clear();
  for (int i = 0; i < 4; i++) {
    qs.push_back(s[i] ? s[i] + 1 : nullptr);
    qns.push_back(s[i] ? Lt[i] - 1 : 0);
  }
}

// KZG::open on a device polynomial; fills x, y, proof
static void kzg_open_device(qg_ctx* ctx, const qg_srs* srs, const Fr* c, size_t L, const Fr& x,
                            qg_kzg_opening* out) {
  fr_export(x, out->x);
  size_t Lt = trimmed_len(ctx, c, L);  // DensePolynomial::from_coefficients_slice trims
  Fr y = Fr::zero();
  G1Affine pi = G1Affine::infinity();
  if (Lt > 0) {
    Fr* s = ctx->scratch_as<Fr>("open_s", Lt);
    {
      QgTimed tm(ctx, "kzg_division");
      suffix_horner(ctx, c, Lt, x, s);
    }
    QG_HIP(hipMemcpyAsync(&y, s, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    // q_i = s_{i+1}, i < Lt - 1; commit(q) (kzg.rs:88-89)
    QG_CHECK(Lt - 1 <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
    pi = msm_device(ctx, srs, s + 1, Lt - 1);
  }
  fr_export(y, out->y);
  g1_export(pi, out->proof_xy, &out->proof_inf);
}

// ---------------------------------------------------------------- sharded opening
// Ranks hold contiguous slices [off, off + L) of a global coefficient vector.
// Suffix-Horner is linear in its carry: the global s_i on a slice equals the
// local scan plus x^(le - i) C, C = global s at the slice end.  C comes from
// one allgather of the per-rank local values T_r = s_local[0].

// s_i += x^(le - i) C for i < le; s_le = C   (pw[k] = x^k)
__global__ void k_sh_carry(Fr* __restrict__ s, size_t le, const Fr* __restrict__ pw, Fr C) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < le) s[i] = s[i] + pw[le - i] * C;
  if (i == le) s[i] = C;
}

// small host values gathered over the communicator (rank order)
static void allgather_host(qg_ctx* ctx, const void* src, size_t bytes, void* dst_all) {
  uint8_t* ds = ctx->scratch_as<uint8_t>("ag_send", bytes);
  uint8_t* dr = ctx->scratch_as<uint8_t>("ag_recv", bytes * (size_t)ctx->world);
  QG_HIP(hipMemcpyAsync(ds, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  comm_allgather_bytes(ctx, ds, dr, bytes);
  QG_HIP(hipMemcpyAsync(dst_all, dr, bytes * (size_t)ctx->world, hipMemcpyDeviceToHost,
                        ctx->stream));
  ctx->sync();
}

// global trimmed length of a vector sliced as [rank * L, rank * L + nloc)
static size_t trimmed_len_global(qg_ctx* ctx, const Fr* a, size_t nloc, size_t L) {
  const uint64_t loc = nloc ? trimmed_len(ctx, a, nloc) : 0;
  const uint64_t mine = loc ? (uint64_t)ctx->rank * L + loc : 0;
  std::vector<uint64_t> all(ctx->world);
  allgather_host(ctx, &mine, sizeof mine, all.data());
  uint64_t m = 0;
  for (uint64_t v : all) m = v > m ? v : m;
  return (size_t)m;
}

// KZG::open of a sharded polynomial (global trimmed length Lt, slices of L):
// every rank gets the same opening; the quotient MSM is sharded.
static void kzg_open_sharded(qg_ctx* ctx, const qg_srs* srs, const Fr* c, size_t L, size_t Lt,
                             const Fr& x, qg_kzg_opening* out) {
  const int world = ctx->world, rank = ctx->rank;
  const size_t off = (size_t)rank * L;
  const size_t le = Lt > off ? std::min(L, Lt - off) : 0;  // this rank's live coefficients
  fr_export(x, out->x);
  Fr* s = ctx->scratch_as<Fr>("open_s", le + 1);
  Fr T = Fr::zero();
  if (le > 0) {
    QgTimed tm(ctx, "kzg_division");
    suffix_horner(ctx, c, le, x, s);
    QG_HIP(hipMemcpyAsync(&T, s, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
  }
  std::vector<Fr> Ts(world);
  allgather_host(ctx, &T, sizeof(Fr), Ts.data());
  // C_r = sum_{r' > r} T_r' x^((r' - r - 1) L);  y = sum_r T_r x^(r L)
  const Fr xL = fpow_small(x, L);
  Fr C = Fr::zero(), y = Fr::zero();
  for (int r = world - 1; r >= 0; r--) {
    if (r == rank) C = y;  // y accumulated over r' > rank so far, in powers of x^L
    y = Ts[r] + xL * y;
  }
  if (le > 0) {
    QgTimed tm(ctx, "kzg_division");
    Fr* pw = ctx->scratch_as<Fr>("open_pw", le + 1);
    const int K = 64;
    hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(le + 1, (size_t)K), ML_BLOCK)), dim3(ML_BLOCK),
                       0, ctx->stream, x, le + 1, K, pw);
    QG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_sh_carry, dim3(div_up(le + 1, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream,
                       s, le, pw, C);
    QG_LAUNCH_CHECK();
  }
  // q_i = s_{i+1} for global i < Lt - 1; this rank's part starts at s + 1
  const size_t qn = (Lt > 0 && Lt - 1 > off) ? std::min(le, Lt - 1 - off) : 0;
  QG_CHECK(qn <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
  const G1Affine pi = msm_device(ctx, srs, s + 1, qn);
  fr_export(y, out->y);
  g1_export(pi, out->proof_xy, &out->proof_inf);
}

// ---------------------------------------------------------------- sharded S polynomial
// S = the window [M, 2M - 1) of h = IDFT_n(Hs), Hs[k] = w^{k(M-1)} / n (F[k] G[-k]
// + F[-k] G[k]) (the replicated s_poly_device, n = 2M), split over W ranks by
// frequency residue.  With k = k2 W + c and i = i1 B + i2 (B = n / W = 2L):
//   F[k2 W + c] = DFT_B(u_c)[k2],  u_c[i2] = w^{i2 c} sum_{i1 < W/2} w_W^{i1 c} f[i1 B + i2]
//   h[i1 B + i2] = sum_c w_W^{-i1 c} w^{-i2 c} IDFT_B(Hs[. W + c])[i2]
// Rank r owns residue c = r: it transforms u_r and the mirror residue (-r mod W,
// for the combine's F[-k] G[-k]), builds G at both residues from the eq
// product formula restricted to the residue (k_eqdft_res), combines, runs one
// B-point inverse, and sends every rank d the L values of h its slice
// S[dL, (d+1)L) = h[M + dL + m] needs (i1 = W/2 + d/2, i2 = (d mod 2) L + m),
// pre-multiplied by w_W^{-i1 c} w^{-i2 c}; one all-to-all, then each rank sums
// the W vectors it received.  Work per rank: 2 B-point DIFs + 1 DIT against
// the replicated path's two 2M-point transforms; the forward input f stays
// the gathered vector (its pre-sum is W/2 multiplies per entry).
// Bit orders as in s_poly_device: DIF outputs bit-reversed within the B block.

// u[i2] = pw[i2] * sum_{i1 < h} cw[i1] f[i1 B + i2]   (cw: w_W^{i1 c} 2^261, pw: w^{i2 c} 2^261)
static constexpr int SP_MAXW = 64;
struct SpConsts {
  L9 v[SP_MAXW];
};
// (f has M entries: W/2 whole blocks for W >= 2; at W = 1 it fills half the one
// block, the rest is the zero padding)
__global__ void k_s_presum(const Fr* __restrict__ f, size_t M, size_t B, uint32_t h, SpConsts cw,
                           const Fr* __restrict__ pw, Fr* __restrict__ u) {
  const size_t i2 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i2 >= B) return;
  R29 acc = R29::zero();
  for (uint32_t i1 = 0; i1 < h; i1++) {
    const size_t g = (size_t)i1 * B + i2;
    if (g < M) acc = red2p29(add29(acc, mul29(to29(f[g]), R29::from_l9(cw.v[i1]))));
  }
  u[i2] = from29(canon29(mul29(acc, to29(pw[i2]))));
}

// G at residue c, bit-reversed within the block, one product-formula level per
// launch (k_eqdft_level restricted to k = c mod W): level t has 2^(lb - t)
// entries e (lb = log2 B), k2 = bitrev(e), factor a_t + z_t w^{(k2 W + c) 2^t}
// = a_t + (z_t w^{c 2^t}) w_B^{k2 2^t}; Q_t[e] = factor Q_{t+1}[e >> 1].
// twBb: w_B^m 2^261 for m < B/2 (w_B^{B/2} = -1) in bit-reversed order
// (ntt_tw_bitrev): w_B^{k2 2^t} is twBb[e >> 1], negated for odd e (as in
// k_eqdft_level).
__global__ void k_eqdft_res(const Fr* __restrict__ qnext, Fr q0, L9 a261, L9 zc261,
                            const Fr* __restrict__ twBb, int lb, int t, Fr* __restrict__ q) {
  const int bits = lb - t;
  const size_t len = (size_t)1 << bits;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= len) return;
  R29 w = to29(twBb[e >> 1]);
  if (e & 1) w = sub29(R29::zero(), w);
  const R29 fct = red2p29(add29(R29::from_l9(a261), mul29(R29::from_l9(zc261), w)));
  const R29 qn = qnext ? to29(qnext[e >> 1]) : to29(q0);
  q[e] = from29(canon29(mul29(fct, qn)));
}

// Hs at residue c in the bit-reversed block order: p -> k2 = bitrev(p); the
// partner of -k is residue m = -c mod W at position ~p (c != 0) or, for c = 0,
// the bit-reversed negation (k_s_combine_br's rule).  Hs = (-1)^c w^{-c} / n
// w_B^{-k2} (F_c G_m' + F_m' G_c): twiBb holds w_B^{-e} 2^261 (e < B/2) in
// bit-reversed order, so w_B^{-k2} = +-twiBb[p >> 1] (the sign from k2's top
// bit, p's low bit; k2's low bit is p's top bit), cst the
// per-residue constant x 2^266 (mul29 of the 2^251-scaled products lands in
// arkworks form).
// At W = 1 the (-1)^k of w^{k(M-1)} = (-1)^k w^{-k} is (-1)^k2, not the
// residue's constant (-1)^c: `alt` negates the odd k2.
__global__ void k_s_combine_res(const Fr* __restrict__ Fc, const Fr* __restrict__ Gc,
                                const Fr* __restrict__ Fm, const Fr* __restrict__ Gm, int c,
                                const Fr* __restrict__ twiBb, int lb, L9 cst, int alt,
                                Fr* __restrict__ H) {
  const size_t B = (size_t)1 << lb;
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= B) return;
  size_t pp;
  if (c != 0) {
    pp = ~p & (B - 1);
  } else {
    pp = 0;
    if (p) {
      const int hb = 63 - __clzll((unsigned long long)p);
      pp = p ^ (((size_t)1 << hb) - 1);
    }
  }
  const bool k2top = lb > 0 && (p & 1), k2low = lb > 0 && ((p >> (lb - 1)) & 1);
  R29 wi = to29(twiBb[p >> 1]);
  if (k2top != (alt && k2low)) wi = sub29(R29::zero(), wi);
  const R29 v = red2p29(add29(mul29(to29(Fc[p]), to29(Gm[pp])), mul29(to29(Fm[pp]), to29(Gc[p]))));
  H[p] = from29(canon29(mul29(mul29(v, red6p29(wi)), R29::from_l9(cst))));
}

// send[d L + m] = K[d] P[i2] Z[i2], i2 = ((M + d L) mod B) + m: (d mod 2) L + m
// for W >= 2 (M = W/2 blocks), L + m at W = 1 (M = L = B/2; `sh` = 1)
// (K: x 2^261, P: x 2^261)
__global__ void k_s_outgoing(const Fr* __restrict__ Z, const Fr* __restrict__ P, SpConsts K,
                             size_t L, uint32_t W, uint32_t sh, Fr* __restrict__ send) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (size_t)W * L) return;
  const uint32_t d = (uint32_t)(i / L);
  const size_t i2 = (size_t)((d + sh) & 1) * L + i % L;
  send[i] = from29(canon29(mul29(mul29(to29(Z[i2]), to29(P[i2])), R29::from_l9(K.v[d]))));
}

// out[m] = sum_s recv[s L + m]
__global__ void k_s_sum_parts(const Fr* __restrict__ recv, size_t L, uint32_t W,
                              Fr* __restrict__ out) {
  const size_t m = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= L) return;
  R29 acc = R29::zero();
  for (uint32_t s = 0; s < W; s++) acc = red2p29(add29(acc, to29(recv[(size_t)s * L + m])));
  out[m] = from29(canon29(acc));
}

static L9 l9_x261(const Fr& mont) {  // Montgomery field element -> (value x 2^261) limbs
  return l9_of29(ml_plain_mul(from_mont(mont), pow2_mod_plain<FrP>(261)));
}

// this rank's slice S[rank L, rank L + L) (L = M / W; the last entry of the last
// slice is h[2M - 1] = 0, past S's M - 1 coefficients).  f: the gathered
// evaluations (M entries, every rank), point: the eq variables (nvars).
static void s_poly_sharded(qg_ctx* ctx, const Fr* f, size_t M, const uint64_t* point,
                           size_t nvars, Fr* S_local) {
  QgTimed tm(ctx, "s_polynomial");
  const uint32_t W = (uint32_t)ctx->world, c = (uint32_t)ctx->rank;
  QG_CHECK(W <= SP_MAXW && (W & (W - 1)) == 0 && M == ((size_t)1 << nvars) && M >= W,
           QG_ERR_UNSUPPORTED, "sharded S polynomial geometry");
  const size_t L = M / W, B = 2 * L;
  int lb = 0;
  while (((size_t)1 << lb) < B) lb++;
  int logn = 0;
  while (((size_t)1 << logn) < 2 * M) logn++;
  QG_CHECK(logn <= 28, QG_ERR_UNSUPPORTED, "S-polynomial NTT beyond 2-adicity");
  Fr *twB, *twiB;
  ntt_twiddles(ctx, lb, &twB, &twiB, "sp_tw");
  const Fr w = root_of_unity(logn), wi = finv(w);
  const Fr wW = fpow_small(w, B);  // w_W = w^(n / W)
  const Fr ninv = finv(from_u64<FrP>((uint64_t)2 * M));
  const uint32_t cm = (W - c) % W;  // mirror residue (-c mod W)
  const int nres = cm == c ? 1 : 2;
  const uint32_t res[2] = {c, cm};
  Fr* Fb = ctx->scratch_as<Fr>("sp_F", 2 * B);
  Fr* Gb = ctx->scratch_as<Fr>("sp_G", 2 * B);
  Fr* tmp = ctx->scratch_as<Fr>("sp_tmp", 2 * B);  // u / pw scratch, then G level ping-pong
  const int K = 64;
  for (int q = 0; q < nres; q++) {
    const uint32_t cc = res[q];
    Fr* Fq = Fb + (size_t)q * B;
    Fr* Gq = Gb + (size_t)q * B;
    // u_cc = w^{i2 cc} sum_i1 w_W^{i1 cc} f[i1 B + i2]
    Fr* pw = tmp + B;
    hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(B, (size_t)K), ML_BLOCK)), dim3(ML_BLOCK), 0,
                       ctx->stream, fpow_small(w, cc), B, K, pw);
    QG_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_fr_to261, dim3(div_up(B, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream, pw, B,
                       F29P<FrP>::TO261);
    QG_LAUNCH_CHECK();
    SpConsts cw{};
    Fr wk = Fr::one();
    const Fr wWc = fpow_small(wW, cc);
    const uint32_t hb = std::max<uint32_t>(1, W / 2);  // input blocks (partial at W = 1)
    for (uint32_t i1 = 0; i1 < hb; i1++) {
      cw.v[i1] = l9_x261(wk);
      wk = wk * wWc;
    }
    hipLaunchKernelGGL(k_s_presum, dim3(div_up(B, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream, f, M,
                       B, hb, cw, pw, tmp);
    QG_LAUNCH_CHECK();
    ntt_run(ctx, true, tmp, B, Fq, twB, "sp_tw", lb, 0, 0, nullptr);
    // G at residue cc: levels above the block collapse into a host constant,
    // then one launch per level t = lb - 1 .. 0 (ping-pong tmp / Gq; nz >= lb
    // whenever W >= 2; at W = 1, nz = lb - 1 and the top level starts from q0 = 1)
    const size_t nz = nvars;
    Fr q0 = Fr::one();
    for (size_t t = nz; t-- > (size_t)lb;) {  // levels with a single entry (t >= lb)
      const Fr zt = fr_import(point + 4 * t);
      q0 = q0 * ((Fr::one() - zt) + zt * fpow_small(w, (uint64_t)cc << t));
    }
    const int top = (int)std::min<size_t>(nz, (size_t)lb);
    const Fr* twBb = ntt_tw_bitrev(ctx, twB, "sp_tw", lb);
    const Fr* qn = nullptr;
    for (int t = top - 1; t >= 0; t--) {
      const Fr zt = fr_import(point + 4 * t);
      const L9 a9 = l9_x261(Fr::one() - zt);
      const L9 z9 = l9_x261(zt * fpow_small(w, (uint64_t)cc << t));
      Fr* dst = (t & 1) == 0 ? Gq : tmp;
      const size_t len = (size_t)1 << (lb - t);
      hipLaunchKernelGGL(k_eqdft_res, dim3(div_up(len, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream,
                         qn, q0, a9, z9, twBb, lb, t, dst);
      QG_LAUNCH_CHECK();
      qn = dst;
    }
  }
  // combine + inverse (own residue), pre-multiplied outgoing vectors, all-to-all, sum
  Fr* H = tmp;
  const Fr* Fm = nres == 2 ? Fb + B : Fb;
  const Fr* Gm = nres == 2 ? Gb + B : Gb;
  Fr cst = fpow_small(wi, c) * ninv;
  if (c & 1) cst = fneg(cst);
  const L9 cst9 = l9_of29(ml_plain_mul(from_mont(cst), pow2_mod_plain<FrP>(266)));
  hipLaunchKernelGGL(k_s_combine_res, dim3(div_up(B, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream, Fb,
                     Gb, Fm, Gm, (int)c, ntt_tw_bitrev(ctx, twiB, "sp_twi", lb), lb, cst9, W == 1 ? 1 : 0,
                     H);
  QG_LAUNCH_CHECK();
  ntt_run(ctx, false, H, B, H, twiB, "sp_twi", lb, 0, 0, nullptr);
  Fr* P = tmp + B;
  hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(B, (size_t)K), ML_BLOCK)), dim3(ML_BLOCK), 0,
                     ctx->stream, fpow_small(wi, c), B, K, P);
  QG_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_fr_to261, dim3(div_up(B, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream, P, B,
                     F29P<FrP>::TO261);
  QG_LAUNCH_CHECK();
  SpConsts Kd{};
  const Fr wWi = finv(wW);
  for (uint32_t d = 0; d < W; d++) {
    const uint64_t i1 = (M + (size_t)d * L) / B;  // W/2 + d/2 for W >= 2, 0 at W = 1
    Kd.v[d] = l9_x261(fpow_small(wWi, (i1 * c) % W));
  }
  Fr* sendb = ctx->scratch_as<Fr>("sp_send", (size_t)W * L);
  Fr* recvb = ctx->scratch_as<Fr>("sp_recv", (size_t)W * L);
  hipLaunchKernelGGL(k_s_outgoing, dim3(div_up((size_t)W * L, ML_BLOCK)), dim3(ML_BLOCK), 0,
                     ctx->stream, H, P, Kd, L, W, W == 1 ? 1u : 0u, sendb);
  QG_LAUNCH_CHECK();
  comm_alltoall_bytes(ctx, sendb, recvb, L * sizeof(Fr));
  hipLaunchKernelGGL(k_s_sum_parts, dim3(div_up(L, ML_BLOCK)), dim3(ML_BLOCK), 0, ctx->stream,
                     recvb, L, W, S_local);
  QG_LAUNCH_CHECK();
}

// MLEvalProof::prove with a communicator: this rank holds poly[rank L, (rank+1) L)
// of the 2^nvars evaluations (L = 2^nvars / world) and the matching SRS shard.
// eq table and the dot product per slice; the S polynomial's transform is split
// by frequency residue over the ranks (s_poly_sharded: the slices are
// allgathered for its forward pre-sum, one all-to-all returns every rank its
// slice of S); its commitment and all four quotient commitments are sharded MSMs.
static void mle_open_sharded(qg_ctx* ctx, const qg_srs* srs, const Fr* dpoly, size_t L,
                             const uint64_t* point, size_t nvars, uint8_t state[32],
                             qg_mle_proof* out) {
  const size_t N = (size_t)1 << nvars;
  QG_CHECK(L * (size_t)ctx->world == N, QG_ERR_UNSUPPORTED,
           "sharded opening needs world * local length == 2^nvars");
  const size_t off = (size_t)ctx->rank * L;
  Fr* dz = ctx->scratch_as<Fr>("mle_z", nvars ? nvars : 1);
  Fr* dpr = ctx->scratch_as<Fr>("mle_pr", N);
  Fr* dfull = ctx->scratch_as<Fr>("mle_full", N);
  fr_upload(ctx, dz, point, nvars);
  eq_table_device(ctx, dz, (uint32_t)nvars, dpr);
  // evaluation: local dot over the slice, summed over ranks
  const Fr part = dot_device(ctx, dpoly, dpr + off, L);
  std::vector<Fr> parts(ctx->world);
  allgather_host(ctx, &part, sizeof(Fr), parts.data());
  Fr evaluation = Fr::zero();
  for (const Fr& v : parts) evaluation = evaluation + v;
  // S: this rank's slice from the residue-split transform (s_poly_sharded) or,
  // with QG_S_REPLICATED=1 (A/B runs), the whole S on every rank
  comm_allgather_bytes(ctx, dpoly, dfull, L * sizeof(Fr));
  const char* rep = getenv("QG_S_REPLICATED");  // read per call: tests toggle it in-process
  const bool replicated = rep && atoi(rep) != 0;
  Fr* Sl = ctx->scratch_as<Fr>("mle_S_local", L);
  size_t Slen = 0;
  if (N > 1) {
    if (replicated) {
      Fr* dS = ctx->scratch_as<Fr>("mle_S", N);
      s_poly_device(ctx, dfull, N, dpr, N, dS, point, nvars);
      QG_HIP(hipMemsetAsync(dS + N - 1, 0, sizeof(Fr), ctx->stream));  // h[2M - 1] = 0
      QG_HIP(hipMemcpyAsync(Sl, dS + off, L * sizeof(Fr), hipMemcpyDeviceToDevice, ctx->stream));
    } else {
      s_poly_sharded(ctx, dfull, N, point, nvars, Sl);
    }
    Slen = trimmed_len_global(ctx, Sl, L, L);
  } else {
    QG_HIP(hipMemsetAsync(Sl, 0, L * sizeof(Fr), ctx->stream));
  }
  const size_t sloc = Slen > off ? std::min(L, Slen - off) : 0;
  QG_CHECK(sloc <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
  G1Affine s_comm = msm_device(ctx, srs, Sl, sloc);
  // transcript: point (Vec<Fr>), evaluation, s_comm; draw r (mlpcs.rs:100-107)
  std::vector<uint8_t> msg(8 + 32 * nvars);
  u64_to_bytes(nvars, msg.data());
  for (size_t i = 0; i < nvars; i++) fr_to_bytes(fr_import(point + 4 * i), msg.data() + 8 + 32 * i);
  transcript_append(state, msg.data(), msg.size());
  uint8_t b32[32], b64[64];
  fr_to_bytes(evaluation, b32);
  transcript_append(state, b32, 32);
  g1_serialize(s_comm, b64);
  transcript_append(state, b64, 64);
  Fr r = transcript_draw_fr(state);
  QG_CHECK(!r.is_zero(), QG_ERR_ASSERT, "challenge r = 0");
  Fr r_inv = finv(r);
  fr_export(evaluation, out->evaluation);
  g1_export(s_comm, out->s_comm_xy, &out->s_comm_inf);
  const size_t Lt = trimmed_len_global(ctx, dpoly, L, L);
  kzg_open_sharded(ctx, srs, dpoly, L, Lt, r, &out->poly_opening);
  kzg_open_sharded(ctx, srs, dpoly, L, Lt, r_inv, &out->poly_opening_inv);
  kzg_open_sharded(ctx, srs, Sl, L, Slen, r, &out->s_opening);
  kzg_open_sharded(ctx, srs, Sl, L, Slen, r_inv, &out->s_opening_inv);
}

struct MleOpenItem {
  const Fr* poly;
  size_t n;
  const uint64_t* point;
  size_t nvars;
  bool unchanged;
  uint64_t id;
  size_t off;
};

// Per-item scratch of a batch of openings (S vectors, quotient vectors, eq
// points) and the per-MSM slots of its MSM batches (msm.hip: partials, owners,
// bucket starts, plan words) stay allocated for the next batch: HyperPlonk
// reuses them trace after trace.  Beyond a working set of OPEN_KEEP items
// (4 OPEN_KEEP MSMs) they are freed when the batch ends (a batch of
// 256 items at 2^20 would otherwise pin ~70-80 GB for the context's lifetime).
static constexpr size_t OPEN_KEEP = 16;
static void open_batch_trim_scratch(qg_ctx* ctx, size_t K) {
  for (size_t k = OPEN_KEEP; k < K; k++) {
    ctx->arena.release("mleb_S#" + std::to_string(k));
    ctx->arena.release("mleb_Sl#" + std::to_string(k));
    ctx->arena.release("mleb_z#" + std::to_string(k));
    ctx->arena.release("open_y#" + std::to_string(k));
  }
  for (size_t j = 4 * OPEN_KEEP; j < 4 * K; j++) {
    ctx->arena.release("open_s#" + std::to_string(j));
    for (const char* m : {"msm_partial#", "msm_owner#", "msm_bstart#", "msm_misc#"})
      ctx->arena.release(m + std::to_string(j));
  }
}

// K openings on a sharded context: mle_open_sharded's data flow, batched the
// way mle_open_batch_device batches the single-context one.  Per item the eq
// table, the local dot, the gathered vector's residue-split S slice and the
// local trimmed lengths are queued; ONE allgather carries every item's dot
// part and local lengths; the S commitments run as ONE MSM batch (one
// allgather of the per-rank partials); the transcript steps run on the host
// in item order; the 4K quotients' local suffix-Horner scans are queued, ONE
// allgather carries their slice-end values T; the carries (x^(le - i) C) are
// applied; the 4K quotient commitments run as ONE MSM batch.  Four exchanges
// per trace instead of ~11 per opening; the proofs and the final transcript
// state equal K successive mle_open_sharded calls (tests/test_gpu_multirank.py).
static void mle_open_batch_sharded(qg_ctx* ctx, const qg_srs* srs,
                                   const std::vector<MleOpenItem>& items, uint8_t state[32],
                                   qg_mle_proof* outs) {
  const size_t K = items.size();
  const size_t W = (size_t)ctx->world, rank = (size_t)ctx->rank;
  for (const MleOpenItem& it : items) {
    QG_CHECK(it.nvars <= 30, QG_ERR_INVALID, "too many variables");
    QG_CHECK(it.n * W == ((size_t)1 << it.nvars), QG_ERR_UNSUPPORTED,
             "sharded opening needs world * local length == 2^nvars");
  }
  // small per-item values of this rank: K dot parts, 2K local trimmed lengths
  const size_t sm_bytes = K * sizeof(Fr) + 2 * K * sizeof(unsigned long long);
  uint8_t* d_sm = ctx->scratch_as<uint8_t>("mlebs_small", sm_bytes);
  Fr* d_part = reinterpret_cast<Fr*>(d_sm);
  unsigned long long* d_len = reinterpret_cast<unsigned long long*>(d_sm + K * sizeof(Fr));
  QG_HIP(hipMemsetAsync(d_sm, 0, sm_bytes, ctx->stream));
  const char* rep = getenv("QG_S_REPLICATED");  // read per call: tests toggle it in-process
  const bool replicated = rep && atoi(rep) != 0;
  std::vector<Fr*> Sl(K);
  for (size_t k = 0; k < K; k++) {
    const MleOpenItem& it = items[k];
    const size_t L = it.n, N = (size_t)1 << it.nvars, off = rank * L;
    Fr* dz = ctx->scratch_as<Fr>("mleb_z#" + std::to_string(k), it.nvars ? it.nvars : 1);
    Fr* dpr = ctx->scratch_as<Fr>("mle_pr", N);
    fr_upload(ctx, dz, it.point, it.nvars);
    eq_table_device(ctx, dz, (uint32_t)it.nvars, dpr);
    dot_to_device(ctx, it.poly, dpr + off, L, d_part + k);
    trim_launch(ctx, it.poly, L, d_len + 2 * k);
    Sl[k] = ctx->scratch_as<Fr>("mleb_Sl#" + std::to_string(k), L);
    if (N > 1) {
      Fr* dfull = ctx->scratch_as<Fr>("mle_full", N);
      comm_allgather_bytes(ctx, it.poly, dfull, L * sizeof(Fr));
      if (replicated) {
        Fr* dS = ctx->scratch_as<Fr>("mle_S", N);
        s_poly_device(ctx, dfull, N, dpr, N, dS, it.point, it.nvars);
        QG_HIP(hipMemsetAsync(dS + N - 1, 0, sizeof(Fr), ctx->stream));  // h[2M - 1] = 0
        QG_HIP(hipMemcpyAsync(Sl[k], dS + off, L * sizeof(Fr), hipMemcpyDeviceToDevice,
                              ctx->stream));
      } else {
        s_poly_sharded(ctx, dfull, N, it.point, it.nvars, Sl[k]);
      }
    } else {
      QG_HIP(hipMemsetAsync(Sl[k], 0, L * sizeof(Fr), ctx->stream));
    }
    trim_launch(ctx, Sl[k], L, d_len + 2 * k + 1);
  }
  // exchange 1: dot parts and local lengths of every rank
  uint8_t* d_all = ctx->scratch_as<uint8_t>("mlebs_small_all", sm_bytes * W);
  comm_allgather_bytes(ctx, d_sm, d_all, sm_bytes);
  std::vector<uint8_t> h_all(sm_bytes * W);
  QG_HIP(hipMemcpyAsync(h_all.data(), d_all, sm_bytes * W, hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  std::vector<Fr> evaluation(K, Fr::zero());
  std::vector<size_t> Lt(K, 0), Slen(K, 0);
  for (size_t r = 0; r < W; r++) {
    const uint8_t* b = h_all.data() + r * sm_bytes;
    const Fr* parts = reinterpret_cast<const Fr*>(b);
    const unsigned long long* lens = reinterpret_cast<const unsigned long long*>(b + K * sizeof(Fr));
    for (size_t k = 0; k < K; k++) {
      evaluation[k] = evaluation[k] + parts[k];
      const size_t L = items[k].n;
      // trimmed_len_global: the largest (rank offset + local length) of a nonzero slice
      if (lens[2 * k]) Lt[k] = std::max(Lt[k], r * L + (size_t)lens[2 * k]);
      if (lens[2 * k + 1]) Slen[k] = std::max(Slen[k], r * L + (size_t)lens[2 * k + 1]);
    }
  }
  // the S commitments: one MSM batch over the local parts of the trimmed S
  std::vector<const Fr*> sp(K);
  std::vector<size_t> sloc(K);
  for (size_t k = 0; k < K; k++) {
    const size_t L = items[k].n, off = rank * L;
    sp[k] = Sl[k];
    sloc[k] = Slen[k] > off ? std::min(L, Slen[k] - off) : 0;
    QG_CHECK(sloc[k] <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
  }
  const std::vector<G1Affine> s_comm = msm_device_batch(ctx, srs, sp, sloc);
  // the transcript steps in item order (mlpcs.rs:100-107)
  std::vector<Fr> xs(4 * K);
  for (size_t k = 0; k < K; k++) {
    const MleOpenItem& it = items[k];
    std::vector<uint8_t> msg(8 + 32 * it.nvars);
    u64_to_bytes(it.nvars, msg.data());
    for (size_t i = 0; i < it.nvars; i++)
      fr_to_bytes(fr_import(it.point + 4 * i), msg.data() + 8 + 32 * i);
    transcript_append(state, msg.data(), msg.size());
    uint8_t b32[32], b64[64];
    fr_to_bytes(evaluation[k], b32);
    transcript_append(state, b32, 32);
    g1_serialize(s_comm[k], b64);
    transcript_append(state, b64, 64);
    const Fr r = transcript_draw_fr(state);
    QG_CHECK(!r.is_zero(), QG_ERR_ASSERT, "challenge r = 0");
    const Fr r_inv = finv(r);
    fr_export(evaluation[k], outs[k].evaluation);
    g1_export(s_comm[k], outs[k].s_comm_xy, &outs[k].s_comm_inf);
    xs[4 * k] = r;
    xs[4 * k + 1] = r_inv;
    xs[4 * k + 2] = r;
    xs[4 * k + 3] = r_inv;
  }
  // the 4K quotients' local scans (kzg_open_sharded, batched): job j = 4k + i
  // scans this rank's le live coefficients into s_j[0..le); T_j = s_j[0]
  const size_t J = 4 * K;
  std::vector<size_t> le(J, 0), glt(J, 0);
  std::vector<Fr*> sq(J, nullptr);
  Fr* d_T = ctx->scratch_as<Fr>("mlebs_T", J);
  QG_HIP(hipMemsetAsync(d_T, 0, J * sizeof(Fr), ctx->stream));
  for (size_t k = 0; k < K; k++) {
    const size_t L = items[k].n, off = rank * L;
    std::vector<ShIn> jobs;
    for (int i = 0; i < 4; i++) {
      const size_t j = 4 * k + i;
      glt[j] = i < 2 ? Lt[k] : Slen[k];
      le[j] = glt[j] > off ? std::min(L, glt[j] - off) : 0;
      sq[j] = ctx->scratch_as<Fr>("open_s#" + std::to_string(j), le[j] + 1);
      if (le[j]) jobs.push_back({i < 2 ? items[k].poly : Sl[k], le[j], xs[j], sq[j]});
    }
    {
      QgTimed tm(ctx, "kzg_division");
      suffix_horner_batch(ctx, jobs);
    }
    for (int i = 0; i < 4; i++) {
      const size_t j = 4 * k + i;
      if (le[j])
        QG_HIP(hipMemcpyAsync(d_T + j, sq[j], sizeof(Fr), hipMemcpyDeviceToDevice, ctx->stream));
    }
  }
  // exchange 2: every rank's T values
  Fr* d_Tall = ctx->scratch_as<Fr>("mlebs_T_all", J * W);
  comm_allgather_bytes(ctx, d_T, d_Tall, J * sizeof(Fr));
  std::vector<Fr> Tall(J * W);
  QG_HIP(hipMemcpyAsync(Tall.data(), d_Tall, J * W * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  // C_rank = sum_{r' > rank} T_r' x^((r' - rank - 1) L);  y = sum_r T_r x^(r L)
  std::vector<Fr> ys(J);
  size_t max_le = 0;
  for (size_t j = 0; j < J; j++) max_le = std::max(max_le, le[j]);
  Fr* pw = ctx->scratch_as<Fr>("open_pw", max_le + 1);
  std::vector<const Fr*> qs(J);
  std::vector<size_t> qn(J);
  for (size_t j = 0; j < J; j++) {
    const size_t L = items[j / 4].n, off = rank * L;
    const Fr x = xs[j], xL = fpow_small(x, L);
    Fr C = Fr::zero(), y = Fr::zero();
    for (size_t r = W; r-- > 0;) {
      if (r == rank) C = y;
      y = Tall[r * J + j] + xL * y;
    }
    ys[j] = y;
    if (le[j] > 0) {
      QgTimed tm(ctx, "kzg_division");
      const int KP = 64;
      hipLaunchKernelGGL(k_powers_ml, dim3(div_up(div_up(le[j] + 1, (size_t)KP), ML_BLOCK)),
                         dim3(ML_BLOCK), 0, ctx->stream, x, le[j] + 1, KP, pw);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_sh_carry, dim3(div_up(le[j] + 1, ML_BLOCK)), dim3(ML_BLOCK), 0,
                         ctx->stream, sq[j], le[j], pw, C);
      QG_LAUNCH_CHECK();
    }
    // q_i = s_{i+1} for global i < Lt - 1; this rank's part starts at s + 1
    qn[j] = (glt[j] > 0 && glt[j] - 1 > off) ? std::min(le[j], glt[j] - 1 - off) : 0;
    QG_CHECK(qn[j] <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
    qs[j] = sq[j] + 1;
  }
  const std::vector<G1Affine> pis = msm_device_batch(ctx, srs, qs, qn);
  for (size_t k = 0; k < K; k++) {
    qg_kzg_opening* o4[4] = {&outs[k].poly_opening, &outs[k].poly_opening_inv,
                             &outs[k].s_opening, &outs[k].s_opening_inv};
    for (int i = 0; i < 4; i++) {
      fr_export(xs[4 * k + i], o4[i]->x);
      fr_export(ys[4 * k + i], o4[i]->y);
      g1_export(pis[4 * k + i], o4[i]->proof_xy, &o4[i]->proof_inf);
    }
  }
  open_batch_trim_scratch(ctx, K);
}

// MLEvalProof::prove (mlpcs.rs:83-124) on a device-resident evaluation vector.
// Two host round trips per opening, both for values the transcript or the
// caller needs: the S commitment and the four quotient commitments.  The
// inner product, the trimmed lengths (DensePolynomial trims, kzg.rs / ipa.rs)
// and the values y are queued into pinned memory and read after those
// synchronizations; the trimmed length of the opened vector is reused while
// the caller guarantees it unchanged (QG_OPEN_UNCHANGED contract, same
// allocation id and offset).
static void mle_open_device(qg_ctx* ctx, const qg_srs* srs, const Fr* dpoly, size_t n,
                            const uint64_t* point, size_t nvars, uint8_t state[32],
                            qg_mle_proof* out, bool unchanged = false, uint64_t poly_id = 0,
                            size_t poly_off = 0) {
  if (ctx->sharded) return mle_open_sharded(ctx, srs, dpoly, n, point, nvars, state, out);
  const size_t N = (size_t)1 << nvars;
  unsigned long long* h_len =
      reinterpret_cast<unsigned long long*>(ctx->pinned_get("mle_len_h", 2 * sizeof(unsigned long long)));
  unsigned long long* d_len = ctx->scratch_as<unsigned long long>("mle_len", 2);
  // trimmed length of the opened vector: queued first (or remembered)
  const std::string lt_key = poly_id ? std::to_string(poly_id) + "+" + std::to_string(poly_off) +
                                           ":" + std::to_string(n) + "="
                                     : std::string();
  std::string& lt_memo = ctx->arena.memo["mle_poly_len"];
  const bool lt_known = unchanged && poly_id && lt_memo.compare(0, lt_key.size(), lt_key) == 0;
  if (!lt_known) {
    trim_launch(ctx, dpoly, n, d_len);
    QG_HIP(hipMemcpyAsync(h_len, d_len, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                          ctx->stream));
  }
  Fr* dz = ctx->scratch_as<Fr>("mle_z", nvars ? nvars : 1);
  Fr* dpr = ctx->scratch_as<Fr>("mle_pr", N);
  fr_upload(ctx, dz, point, nvars);
  // P_r coefficients = eq table (mlpcs.rs:68-78)
  eq_table_device(ctx, dz, (uint32_t)nvars, dpr);
  // evaluation = <poly, P_r> over the common prefix (mlpcs.rs:91-94)
  Fr* d_eval = ctx->scratch_as<Fr>("mle_eval", 1);
  Fr* h_eval = reinterpret_cast<Fr*>(ctx->pinned_get("mle_eval_h", sizeof(Fr)));
  dot_to_device(ctx, dpoly, dpr, n < N ? n : N, d_eval);
  QG_HIP(hipMemcpyAsync(h_eval, d_eval, sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  // S polynomial (mlpcs.rs:95-97) and its trimmed length
  const size_t M = n > N ? n : N;
  const size_t Sn = M > 1 ? M - 1 : 0;
  Fr* dS = ctx->scratch_as<Fr>("mle_S", Sn ? Sn : 1);
  if (Sn) s_poly_device(ctx, dpoly, n, dpr, N, dS, point, nvars, unchanged, poly_id, poly_off);
  trim_launch(ctx, dS, Sn, d_len + 1);
  QG_HIP(hipMemcpyAsync(h_len + 1, d_len + 1, sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        ctx->stream));
  // its commitment: over all Sn coefficients when they fit the SRS (trailing
  // zeros add nothing), else the trimmed length first (the degree check)
  size_t s_msm = Sn;
  if (Sn > srs->n) {
    ctx->sync();
    s_msm = (size_t)h_len[1];
    QG_CHECK(s_msm <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
  }
  G1Affine s_comm = msm_device(ctx, srs, dS, s_msm);
  ctx->sync();  // (drained already unless the MSM was empty)
  const Fr evaluation = *h_eval;
  const size_t Slen = (size_t)h_len[1];
  size_t Lt = 0;
  if (lt_known) {
    Lt = (size_t)std::stoull(lt_memo.substr(lt_key.size()));
  } else {
    Lt = (size_t)h_len[0];
    lt_memo = poly_id ? lt_key + std::to_string(Lt) : std::string();
  }
  // transcript: point (Vec<Fr>), evaluation, s_comm; draw r (mlpcs.rs:100-107)
  std::vector<uint8_t> msg(8 + 32 * nvars);
  u64_to_bytes(nvars, msg.data());
  for (size_t i = 0; i < nvars; i++) fr_to_bytes(fr_import(point + 4 * i), msg.data() + 8 + 32 * i);
  transcript_append(state, msg.data(), msg.size());
  uint8_t b32[32], b64[64];
  fr_to_bytes(evaluation, b32);
  transcript_append(state, b32, 32);
  g1_serialize(s_comm, b64);
  transcript_append(state, b64, 64);
  Fr r = transcript_draw_fr(state);
  QG_CHECK(!r.is_zero(), QG_ERR_ASSERT, "challenge r = 0");
  Fr r_inv = finv(r);
  fr_export(evaluation, out->evaluation);
  g1_export(s_comm, out->s_comm_xy, &out->s_comm_inf);
  // four KZG openings (mlpcs.rs:108-113): the four quotients first, then their
  // commitments as one MSM batch (shared reduction launches)
  qg_kzg_opening* outs[4] = {&out->poly_opening, &out->poly_opening_inv, &out->s_opening,
                             &out->s_opening_inv};
  const Fr* polys[4] = {dpoly, dpoly, dS, dS};
  const size_t lts[4] = {Lt, Lt, Slen, Slen};
  const Fr xs[4] = {r, r_inv, r, r_inv};
  std::vector<const Fr*> qs;
  std::vector<size_t> qns;
  Fr* h_y = reinterpret_cast<Fr*>(ctx->pinned_get("open_y_h", 4 * sizeof(Fr)));
  kzg_quotients_batch(ctx, srs, polys, lts, xs, outs, qs, qns, h_y);
  const std::vector<G1Affine> pis = msm_device_batch(ctx, srs, qs, qns);
  ctx->sync();  // (drained already unless every quotient was empty)
  for (int i = 0; i < 4; i++) {
    fr_export(h_y[i], outs[i]->y);
    g1_export(pis[i], outs[i]->proof_xy, &outs[i]->proof_inf);
  }
}

// K ML openings with the transcript steps in item order — the same proofs and
// final state as K successive mle_open_device calls — restructured around the
// protocol's data flow (mlpcs.rs:83-124): S, its commitment, the evaluation
// and the trimmed lengths depend on the polynomial and the point only, and
// the transcript absorbs no quotient commitment, so
//   1. every item's evaluation, S polynomial and trimmed lengths (queued),
//   2. the K S commitments as ONE MSM batch (one synchronization),
//   3. the K transcript steps on the host (append point, evaluation, s_comm;
//      draw r),
//   4. the 4K quotients and their commitments as ONE MSM batch.
// Inside a batch the bucketing of MSM i + 1 runs on the side stream beside
// MSM i's accumulation, and the batch pays one set of reduction launches and
// one host round trip (msm.hip).  Sharded contexts open item by item.

static void mle_open_batch_device(qg_ctx* ctx, const qg_srs* srs,
                                  const std::vector<MleOpenItem>& items, uint8_t state[32],
                                  qg_mle_proof* outs) {
  const size_t K = items.size();
  // QG_OPEN_BATCH_SHARDED=0: a sharded context opens item by item (A/B runs)
  const char* sb = getenv("QG_OPEN_BATCH_SHARDED");
  if (ctx->sharded && K > 1 && !(sb && atoi(sb) == 0))
    return mle_open_batch_sharded(ctx, srs, items, state, outs);
  if (ctx->sharded || K <= 1) {
    for (size_t k = 0; k < K; k++)
      mle_open_device(ctx, srs, items[k].poly, items[k].n, items[k].point, items[k].nvars, state,
                      &outs[k], items[k].unchanged, items[k].id, items[k].off);
    return;
  }
  unsigned long long* h_len = reinterpret_cast<unsigned long long*>(
      ctx->pinned_get("mleb_len_h", 2 * K * sizeof(unsigned long long)));
  unsigned long long* d_len = ctx->scratch_as<unsigned long long>("mleb_len", 2 * K);
  Fr* h_eval = reinterpret_cast<Fr*>(ctx->pinned_get("mleb_eval_h", K * sizeof(Fr)));
  Fr* d_eval = ctx->scratch_as<Fr>("mleb_eval", K);
  QG_HIP(hipMemsetAsync(d_len, 0, 2 * K * sizeof(unsigned long long), ctx->stream));
  // the opened vectors' trimmed lengths: remembered for the QG_OPEN_UNCHANGED
  // contract exactly as K successive mle_open_device calls would (the memo
  // holds the last opened vector's key and length): item k reuses it when
  // flagged and item k - 1 (item 0: the memo from before this call) opened
  // the same vector
  std::string& lt_memo = ctx->arena.memo["mle_poly_len"];
  const std::string memo_in = lt_memo;
  std::vector<std::string> lt_key(K);
  std::vector<char> lt_known(K, 0);
  std::vector<Fr*> dS(K, nullptr);
  std::vector<size_t> Sn(K, 0), s_msm(K, 0);
  bool s_trim_first = false;
  for (size_t k = 0; k < K; k++) {
    const MleOpenItem& it = items[k];
    QG_CHECK(it.nvars <= 30, QG_ERR_INVALID, "too many variables");
    const size_t N = (size_t)1 << it.nvars;
    lt_key[k] = it.id ? std::to_string(it.id) + "+" + std::to_string(it.off) + ":" +
                            std::to_string(it.n) + "="
                      : std::string();
    lt_known[k] = it.unchanged && it.id &&
                  (k == 0 ? memo_in.compare(0, lt_key[k].size(), lt_key[k]) == 0
                          : lt_key[k - 1] == lt_key[k]);
    if (!lt_known[k]) trim_launch(ctx, it.poly, it.n, d_len + 2 * k);
    Fr* dz = ctx->scratch_as<Fr>("mleb_z#" + std::to_string(k), it.nvars ? it.nvars : 1);
    Fr* dpr = ctx->scratch_as<Fr>("mle_pr", N);
    fr_upload(ctx, dz, it.point, it.nvars);
    eq_table_device(ctx, dz, (uint32_t)it.nvars, dpr);
    dot_to_device(ctx, it.poly, dpr, it.n < N ? it.n : N, d_eval + k);
    const size_t M = it.n > N ? it.n : N;
    Sn[k] = M > 1 ? M - 1 : 0;
    dS[k] = ctx->scratch_as<Fr>("mleb_S#" + std::to_string(k), Sn[k] ? Sn[k] : 1);
    if (Sn[k])
      s_poly_device(ctx, it.poly, it.n, dpr, N, dS[k], it.point, it.nvars, it.unchanged, it.id,
                    it.off);
    trim_launch(ctx, dS[k], Sn[k], d_len + 2 * k + 1);
    s_msm[k] = Sn[k];
    s_trim_first = s_trim_first || Sn[k] > srs->n;
  }
  QG_HIP(hipMemcpyAsync(h_len, d_len, 2 * K * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                        ctx->stream));
  QG_HIP(hipMemcpyAsync(h_eval, d_eval, K * sizeof(Fr), hipMemcpyDeviceToHost, ctx->stream));
  if (s_trim_first) {  // an S longer than the SRS: its trimmed length decides
    ctx->sync();
    for (size_t k = 0; k < K; k++)
      if (Sn[k] > srs->n) {
        s_msm[k] = (size_t)h_len[2 * k + 1];
        QG_CHECK(s_msm[k] <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
      }
  }
  std::vector<const Fr*> sp(dS.begin(), dS.end());
  const std::vector<G1Affine> s_comm = msm_device_batch(ctx, srs, sp, s_msm);
  ctx->sync();  // (drained already unless every MSM was empty)
  // the transcript steps in item order (mlpcs.rs:100-107)
  std::vector<Fr> rs(K), rinv(K);
  std::vector<size_t> Lt(K);
  for (size_t k = 0; k < K; k++) {
    const MleOpenItem& it = items[k];
    if (lt_known[k])
      Lt[k] = k == 0 ? (size_t)std::stoull(memo_in.substr(lt_key[k].size())) : Lt[k - 1];
    else
      Lt[k] = (size_t)h_len[2 * k];
    lt_memo = it.id ? lt_key[k] + std::to_string(Lt[k]) : std::string();
    const Fr evaluation = h_eval[k];
    std::vector<uint8_t> msg(8 + 32 * it.nvars);
    u64_to_bytes(it.nvars, msg.data());
    for (size_t i = 0; i < it.nvars; i++)
      fr_to_bytes(fr_import(it.point + 4 * i), msg.data() + 8 + 32 * i);
    transcript_append(state, msg.data(), msg.size());
    uint8_t b32[32], b64[64];
    fr_to_bytes(evaluation, b32);
    transcript_append(state, b32, 32);
    g1_serialize(s_comm[k], b64);
    transcript_append(state, b64, 64);
    rs[k] = transcript_draw_fr(state);
    QG_CHECK(!rs[k].is_zero(), QG_ERR_ASSERT, "challenge r = 0");
    rinv[k] = finv(rs[k]);
    fr_export(evaluation, outs[k].evaluation);
    g1_export(s_comm[k], outs[k].s_comm_xy, &outs[k].s_comm_inf);
  }
  // every item's four quotients (mlpcs.rs:108-113), then all 4K commitments
  Fr* h_y = reinterpret_cast<Fr*>(ctx->pinned_get("mleb_y_h", 4 * K * sizeof(Fr)));
  std::vector<const Fr*> qs_all;
  std::vector<size_t> qns_all;
  for (size_t k = 0; k < K; k++) {
    qg_kzg_opening* o4[4] = {&outs[k].poly_opening, &outs[k].poly_opening_inv,
                             &outs[k].s_opening, &outs[k].s_opening_inv};
    const Fr* polys[4] = {items[k].poly, items[k].poly, dS[k], dS[k]};
    const size_t slen = (size_t)h_len[2 * k + 1];
    const size_t lts[4] = {Lt[k], Lt[k], slen, slen};
    const Fr xs[4] = {rs[k], rinv[k], rs[k], rinv[k]};
    std::vector<const Fr*> qs;
    std::vector<size_t> qns;
    kzg_quotients_batch(ctx, srs, polys, lts, xs, o4, qs, qns, h_y + 4 * k, k);
    qs_all.insert(qs_all.end(), qs.begin(), qs.end());
    qns_all.insert(qns_all.end(), qns.begin(), qns.end());
  }
  const std::vector<G1Affine> pis = msm_device_batch(ctx, srs, qs_all, qns_all);
  ctx->sync();  // (drained already unless every quotient was empty)
  for (size_t k = 0; k < K; k++) {
    qg_kzg_opening* o4[4] = {&outs[k].poly_opening, &outs[k].poly_opening_inv,
                             &outs[k].s_opening, &outs[k].s_opening_inv};
    for (int i = 0; i < 4; i++) {
      fr_export(h_y[4 * k + i], o4[i]->y);
      g1_export(pis[4 * k + i], o4[i]->proof_xy, &o4[i]->proof_inf);
    }
  }
  open_batch_trim_scratch(ctx, K);
}

}  // namespace qg

extern "C" {

int qg_inner_product(qg_ctx* ctx, const uint64_t* f, size_t nf, const uint64_t* g, size_t ng,
                     uint64_t out[4]) {
  if (!ctx || (!f && nf) || (!g && ng) || !out) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    size_t n = nf < ng ? nf : ng;
    Fr* df = ctx->scratch_as<Fr>("ip_f", n ? n : 1);
    Fr* dg = ctx->scratch_as<Fr>("ip_g", n ? n : 1);
    fr_upload(ctx, df, f, n);
    fr_upload(ctx, dg, g, n);
    fr_export(dot_device(ctx, df, dg, n), out);
  });
}

int qg_s_polynomial(qg_ctx* ctx, const uint64_t* f, size_t nf, const uint64_t* g, size_t ng,
                    uint64_t* out) {
  if (!ctx || (!f && nf) || (!g && ng) || (!out && (nf > 1 || ng > 1))) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    const size_t M = nf > ng ? nf : ng;
    if (M <= 1) return;
    Fr* df = ctx->scratch_as<Fr>("sp_f", nf ? nf : 1);
    Fr* dg = ctx->scratch_as<Fr>("sp_g", ng ? ng : 1);
    Fr* dS = ctx->scratch_as<Fr>("sp_S", M - 1);
    fr_upload(ctx, df, f, nf);
    fr_upload(ctx, dg, g, ng);
    s_poly_device(ctx, df, nf, dg, ng, dS);
    fr_download(ctx, out, dS, M - 1);
    ctx->sync();
  });
}

int qg_kzg_open(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n, const uint64_t x[4],
                qg_kzg_opening* out) {
  if (!ctx || !srs || (!poly && n) || !x || !out) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    Fr* d = ctx->scratch_as<Fr>("open_in", n ? n : 1);
    fr_upload(ctx, d, poly, n);
    kzg_open_device(ctx, srs, d, n, fr_import(x), out);
  });
}

int qg_mle_open(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n,
                const uint64_t* point, size_t nvars, uint8_t state[32], qg_mle_proof* out) {
  if (!ctx || !srs || (!poly && n) || (!point && nvars) || !state || !out) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars <= 30, QG_ERR_INVALID, "too many variables");
    QG_HIP(hipSetDevice(ctx->device));
    Fr* dpoly = ctx->scratch_as<Fr>("mle_poly", n ? n : 1);
    fr_upload(ctx, dpoly, poly, n);
    mle_open_device(ctx, srs, dpoly, n, point, nvars, state, out);
  });
}

int qg_mle_open_dev(qg_ctx* ctx, const qg_srs* srs, const qg_buf* poly, size_t n,
                    const uint64_t* point, size_t nvars, uint8_t state[32], qg_mle_proof* out) {
  if (!ctx || !srs || !poly || n > poly->n || (!point && nvars) || !state || !out)
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars <= 30, QG_ERR_INVALID, "too many variables");
    QG_HIP(hipSetDevice(ctx->device));
    mle_open_device(ctx, srs, poly->d, n, point, nvars, state, out);
  });
}

int qg_mle_open_batch_dev(qg_ctx* ctx, const qg_srs* srs, const qg_mle_open_item* items,
                          size_t k, uint8_t state[32], qg_mle_proof* outs) {
  if (!ctx || !srs || (!items && k) || !state || (!outs && k)) return QG_ERR_INVALID;
  for (size_t i = 0; i < k; i++)
    if (!items[i].poly || items[i].n > items[i].poly->n || (!items[i].point && items[i].nvars) ||
        items[i].nvars > 30 || (items[i].flags & ~(uint32_t)QG_OPEN_UNCHANGED))
      return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(k <= 256, QG_ERR_UNSUPPORTED, "too many openings in one batch (at most 256)");
    QG_HIP(hipSetDevice(ctx->device));
    std::vector<MleOpenItem> v(k);
    for (size_t i = 0; i < k; i++)
      v[i] = {items[i].poly->d, items[i].n, items[i].point, items[i].nvars,
              (items[i].flags & QG_OPEN_UNCHANGED) != 0, items[i].poly->alloc_id,
              items[i].poly->base_off};
    mle_open_batch_device(ctx, srs, v, state, outs);
  });
}

int qg_mle_open_dev_ex(qg_ctx* ctx, const qg_srs* srs, const qg_buf* poly, size_t n,
                       const uint64_t* point, size_t nvars, uint8_t state[32], uint32_t flags,
                       qg_mle_proof* out) {
  if (!ctx || !srs || !poly || n > poly->n || (!point && nvars) || !state || !out ||
      (flags & ~(uint32_t)QG_OPEN_UNCHANGED))
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(nvars <= 30, QG_ERR_INVALID, "too many variables");
    QG_HIP(hipSetDevice(ctx->device));
    mle_open_device(ctx, srs, poly->d, n, point, nvars, state, out,
                    (flags & QG_OPEN_UNCHANGED) != 0, poly->alloc_id, poly->base_off);
  });
}

}  // extern "C"
