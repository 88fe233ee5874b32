// Pippenger MSM over BN254 G1 for gfx950 — replaces
// `E::G1::msm_unchecked(&g1_points_affine, polynomial)` at pcs/src/kzg.rs:72
// (ark-ec 0.5.0 VariableBaseMSM) and the SRS handling of KZG::commit
// (kzg.rs:61-73) / KZG::trusted_setup (kzg.rs:35-59).
//
// Design (MI355X-first):
//  * The SRS lives in HBM as W window-shifted tables table[w][i] = 2^(c*w) * P_i,
//    one 128-B row per point (x, y and p - y in 9 x 29-bit limbs + flags, so a
//    negative digit costs no arithmetic).  288 GB of HBM makes this affordable
//    (2^24 bases, c = 20: 13 tables, 27.9 GB, built once per SRS outside any
//    commitment) and removes the serial window-combination doublings: every
//    signed c-bit digit of every scalar lands in ONE shared set of 2^(c-1)
//    buckets.
//  * Bucketing is a two-pass LDS radix sort (pass A by bucket-high bits over
//    512-scalar tiles, pass B by bucket-low bits within 8192-entry chunks);
//    digits come from the canonical scalars by funnel shifts.
//  * Accumulation is load-balanced: the bucket-sorted entries are cut into
//    flat chunks of L entries, one thread per chunk, so skewed digit
//    distributions (small witness values, the short top window) do not
//    serialize on one lane.  Mixed XYZZ + affine additions (8M + 2S), no
//    inversions; a raw partial is flushed at every bucket boundary.
//  * Bucket reduction sum_j (j+1) B_j: each lane sums its buckets' partial
//    slots on the fly with running sums from the top, then shuffle folds
//    (suffix scan + tree) and three quad-cooperative folds of 16.
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "curve29.h"

using namespace qg;

namespace qg {

static constexpr int MSM_BLOCK = 256;

// Window size for an SRS of n bases.  Cost model in bucket-addition units:
// n * ceil(255 / c) accumulations + ~12 per bucket for bucketing and the
// reduction (fitted to MI355X runs: 2^24 c = 20 vs 22, 2^22 c = 20 vs 17 / 19).
// Windows whose top digit covers few bits (k = 254 - c (W - 1), scalars <
// 2^254) send n / 2^k entries to each of 2^k buckets (skewed combine):
// excluded when that exceeds 4096.  Gives c = 17 at 2^20, 20 at 2^21..2^24.
static int msm_window_bits(size_t n) {
  int best = 4;
  double best_cost = 1e300;
  for (int c = 4; c <= 22; c++) {
    const int W = (255 + c - 1) / c;
    const int k = 254 - c * (W - 1);
    if (k < 30 && (n >> k) > 4096) continue;
    const double cost = (double)n * W + 12.0 * (double)((size_t)1 << (c - 1));
    if (cost < best_cost) {
      best_cost = cost;
      best = c;
    }
  }
  return best;
}

// canonical words of a Montgomery-form scalar, x 2^-256 mod r: the 29-bit
// Montgomery reduction (mul29 by the plain integer 2^5: 2^5 2^-261 = 2^-256),
// no 32-bit carry chains
QG_DEV Fr fr_canon29(const Fr& x) {
  F29<FrP> k = F29<FrP>::zero();
  k.l[0] = 32;
  return from29(canon29(mul29(to29(x), k)));
}

// signed c-bit digit decomposition of a CANONICAL scalar (8 words), emit(w,
// bucket, neg) for nonzero digits.  The window walks the words by funnel
// shifts (v_alignbit), all register-resident: no dynamically indexed array
// (which would live in scratch memory).  c < 32.
template <class Emit>
QG_DEV void for_each_digit(const Fr& canon, int c, int W, Emit&& emit) {
  uint32_t v[8];
#pragma unroll
  for (int i = 0; i < 8; i++) v[i] = canon.v[i];
  const uint32_t mask = (1u << c) - 1u;
  const uint32_t half = 1u << (c - 1);
  const uint32_t full = 1u << c;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    const uint32_t d = (v[0] & mask) + carry;
    if (d > half) {
      carry = 1;
      const uint32_t mag = full - d;  // digit = d - 2^c < 0
      if (mag) emit(w, mag - 1, true);
    } else {
      carry = 0;
      if (d) emit(w, d - 1, false);
    }
#pragma unroll
    for (int i = 0; i < 7; i++) v[i] = __builtin_amdgcn_alignbit(v[i + 1], v[i], (uint32_t)c);
    v[7] >>= c;
  }
}

// XCD-aware tile order: workgroup b runs on XCD b % 8 (placement is a speed
// hint only, never assumed for correctness), so tile t = start(b % 8) + b / 8
// gives every XCD one contiguous range of tiles.  The runs that neighbouring
// tiles write into one group / bucket region are then adjacent in the same
// L2, which merges their partial lines before write-back.  A bijection of
// [0, G).
QG_DEV uint32_t xcd_tile(uint32_t b, uint32_t G) {
  const uint32_t x = b & 7u, q = G >> 3, r = G & 7u;
  return x * q + (x < r ? x : r) + (b >> 3);
}

// ---- bucketing: two-pass LDS-histogram radix sort ------------------------
// Bucket id b (BB = c-1 bits) = (g << LO) | l.  Pass A partitions digits by the
// high part g with per-block LDS histograms (no per-digit global atomics);
// pass B sorts every group by l in chunks of SORT_CHUNK entries, so a heavy
// group (skewed scalars, the short top window) spreads over many blocks.
static constexpr int SORT_BLOCK = 256;
static constexpr int SORT_TILE_MAX = 1024;                  // scalars per block (pass A)
static constexpr size_t SORT_LDS_A = 72 * 1024;             // LDS budget for staged entries (2 blocks/CU)
#ifndef QG_SORT_CHUNK
#define QG_SORT_CHUNK 8192
#endif
static constexpr int SORT_CHUNK = QG_SORT_CHUNK;            // entries per block (pass B)

// ---- cross-stream hand-over guard (msm_device_batch) ----------------------
// A batch on the side streams hands data over by events only: the scalars
// from the context stream to the side streams, the partial sums back.  Each
// hand-over is also checked on the device: the producer stream writes this
// batch's generation into a tag word (k_handover_tag, after its last producer
// kernel); every block of the consumer kernels reads the tag when it starts
// and sets an error bit if it does not hold the generation yet, i.e. if the
// block started before the producer stream reached the tag.  hv[0]: tag of the
// scalars, hv[1]: error bits (1 = scalars, 2 = partials), hv[2 + p]: tag of
// side stream p's last accumulation.  The host reads hv[1] with the results
// and recomputes the batch in stream order if it is not 0 (counted as
// `msm_handover_violation`).
__global__ void k_handover_tag(uint32_t* hv, uint32_t w, uint32_t gen, uint32_t clear) {
  if (threadIdx.x == 0) {
    if (clear) hv[1] = hv[2] = hv[3] = 0u;
    hv[w] = gen;
  }
}

QG_DEV void msm_handover_check(uint32_t* hv, uint32_t w0, uint32_t nw, uint32_t gen, uint32_t bit) {
  if (hv == nullptr || threadIdx.x != 0) return;
  for (uint32_t w = w0; w < w0 + nw; w++)
    if (__hip_atomic_load(hv + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen) {
      atomicOr(hv + 1, bit);
      return;
    }
}

// Pass A histogram; also writes every scalar's canonical words (`canon`), so
// the scatter pass reads them without a second Montgomery reduction.
// hv != null: the scalars came from another stream (hand-over guard above)
// wsel >= 0: only window wsel's digits (one-shot bases, msm_oneshot_local);
// canon_ready: `canon` already holds these scalars' canonical words (the
// one-shot windows after the first), read instead of recomputed and rewritten
__global__ void __launch_bounds__(SORT_BLOCK)
    k_sortA_hist(const Fr* __restrict__ scalars, size_t n, int c, int W, int LO, int H,
                 uint32_t nblk, uint32_t tile, uint32_t* __restrict__ hrow, Fr* __restrict__ canon,
                 uint32_t* hv, uint32_t gen, int wsel, int canon_ready) {
  extern __shared__ uint32_t hist[];
  msm_handover_check(hv, 0, 1, gen, 1u);
  for (int g = threadIdx.x; g < H; g += blockDim.x) hist[g] = 0;
  __syncthreads();
  const uint32_t tb = xcd_tile(blockIdx.x, nblk);
  const size_t base = (size_t)tb * tile;
  const size_t end = base + tile < n ? base + tile : n;
  static_assert(SORT_TILE_MAX % SORT_BLOCK == 0, "pass-A tile must split evenly over the block");
  for (size_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    Fr s;
    if (canon_ready) {
      s = canon[i];
    } else {
      s = fr_canon29(scalars[i]);
      canon[i] = s;
    }
    for_each_digit(s, c, W, [&](int w, uint32_t b, bool) {
      if (wsel < 0 || w == wsel) atomicAdd(&hist[b >> LO], 1u);
    });
  }
  __syncthreads();
  // row-major (tile, group): one contiguous row per block; transposed for the scan
  for (int g = threadIdx.x; g < H; g += blockDim.x) hrow[(size_t)tb * H + g] = hist[g];
}

// out[c][r] = in[r][c] for a rows x cols u32 matrix (32 x 32 LDS tiles)
__global__ void __launch_bounds__(256)
    k_transpose32(const uint32_t* __restrict__ in, uint32_t rows, uint32_t cols,
                  uint32_t* __restrict__ out) {
  __shared__ uint32_t tile[32][33];
  const uint32_t c0 = blockIdx.x * 32, r0 = blockIdx.y * 32;
  const uint32_t tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (uint32_t k = ty; k < 32; k += 8)
    if (r0 + k < rows && c0 + tx < cols) tile[k][tx] = in[(size_t)(r0 + k) * cols + c0 + tx];
  __syncthreads();
  for (uint32_t k = ty; k < 32; k += 8)
    if (c0 + k < cols && r0 + tx < rows) out[(size_t)(c0 + k) * rows + r0 + tx] = tile[tx][k];
}

// Block-local exclusive scan of n <= 4 * SORT_BLOCK counts in LDS (in place).
// Each thread owns `per` consecutive counts; the thread totals are scanned
// within the wave by shuffles, the 4 wave totals through LDS: two barriers
// (a Hillis-Steele scan over the block took 2 x 8).
__device__ void lds_exscan(uint32_t* a, int n, uint32_t* tmp /* >= SORT_BLOCK / 64 words */) {
  const int per = (n + SORT_BLOCK - 1) / SORT_BLOCK;
  const int b = threadIdx.x * per;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t tot = 0;
  for (int k = 0; k < per; k++)
    if (b + k < n) tot += a[b + k];
  uint32_t inc = tot;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(inc, d, 64);
    if (lane >= d) inc += y;
  }
  if (lane == 63) tmp[wid] = inc;
  __syncthreads();
  uint32_t run = inc - tot;
  for (int w = 0; w < wid; w++) run += tmp[w];
  for (int k = 0; k < per; k++) {
    if (b + k < n) {
      const uint32_t v = a[b + k];
      a[b + k] = run;
      run += v;
    }
  }
  __syncthreads();
}

// largest g with off[g] <= p (off ascending, n entries)
__device__ __forceinline__ int lds_upper(const uint32_t* off, int n, uint32_t p) {
  int lo = 0, hi = n;
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (off[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

// Pass A scatter: digits of the block's tile are bucketed by group in LDS
// (entry + its bucket), then written out as contiguous per-group runs
// (coalesced stores) through a per-block base table, no per-element search.
// The block's counts and global offsets are contiguous rows (hrow / orow).
// Output per digit: the table entry (u32) and the bucket's low LO bits (u16).
// wsel >= 0: only window wsel's digits, entry = the base's row in the one
// table of one-shot bases (no window offset)
__global__ void __launch_bounds__(SORT_BLOCK)
    k_sortA_scatter(const Fr* __restrict__ canon, size_t n, size_t N, size_t off, int c, int W, int LO,
                    int H,
                    uint32_t nblk, uint32_t tile, const uint32_t* __restrict__ hrow,
                    const uint32_t* __restrict__ orow, uint32_t* __restrict__ tmp_e,
                    uint16_t* __restrict__ tmp_l, int wsel) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* ent = reinterpret_cast<uint32_t*>(smem);
  uint32_t* bkt = ent + (size_t)tile * (wsel < 0 ? W : 1);
  uint32_t* loff = bkt + (size_t)tile * (wsel < 0 ? W : 1);
  uint32_t* cur = loff + H;
  uint32_t* gb = cur + H;
  uint32_t* scr = gb + H;
  (void)scr;
  const uint32_t tb = xcd_tile(blockIdx.x, nblk);
  const size_t base = (size_t)tb * tile;
  const size_t end = base + tile < n ? base + tile : n;
  // the thread's scalars (tile <= SORT_TILE_MAX) are loaded first: their round
  // trip overlaps the row loads below
  constexpr int PER = SORT_TILE_MAX / SORT_BLOCK;
  Fr sv[PER];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const size_t i = base + threadIdx.x + (size_t)j * SORT_BLOCK;
    if (i < end) sv[j] = canon[i];
  }
  // rows prepared by k_sortA_rows: the tile's local run starts and global bases
  for (int g = threadIdx.x; g < H; g += blockDim.x) {
    loff[g] = hrow[(size_t)tb * H + g];
    gb[g] = orow[(size_t)tb * H + g];
    cur[g] = 0;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const size_t i = base + threadIdx.x + (size_t)j * SORT_BLOCK;
    if (i >= end) break;
    for_each_digit(sv[j], c, W, [&](int w, uint32_t b, bool neg) {
      if (wsel >= 0 && w != wsel) return;
      const uint32_t g = b >> LO;
      const uint32_t slot = loff[g] + atomicAdd(&cur[g], 1u);
      const size_t row = (wsel < 0 ? (size_t)w * N : 0) + off + i;
      ent[slot] = (uint32_t)row | (neg ? 0x80000000u : 0u);
      bkt[slot] = b;
    });
  }
  __syncthreads();
  const uint32_t total = loff[H - 1] + cur[H - 1];
  const uint32_t lmask = (1u << LO) - 1u;
  for (uint32_t p = threadIdx.x; p < total; p += blockDim.x) {
    const uint32_t b = bkt[p];
    const uint32_t dst = gb[b >> LO] + p;
    tmp_e[dst] = ent[p];
    tmp_l[dst] = (uint16_t)(b & lmask);
  }
}

// per tile row (one block each): hrow <- exclusive scan of the tile's group
// counts (its local run starts), orow <- global offset - local start (the base
// that the scatter adds to an LDS position)
__global__ void __launch_bounds__(SORT_BLOCK)
    k_sortA_rows(uint32_t* __restrict__ hrow, uint32_t* __restrict__ orow, int H) {
  __shared__ uint32_t a[4 * SORT_BLOCK], scr[SORT_BLOCK];
  const size_t r = (size_t)blockIdx.x * H;
  for (int g = threadIdx.x; g < H; g += blockDim.x) a[g] = hrow[r + g];
  __syncthreads();
  lds_exscan(a, H, scr);
  for (int g = threadIdx.x; g < H; g += blockDim.x) {
    hrow[r + g] = a[g];
    orow[r + g] -= a[g];
  }
}

// groups -> chunks (single block): gstart[g] = goff[g*nblk], chunk bases, chunk->group map;
// misc[0] = chunk count, and the words the bucket scan accumulates into start
// here (no fill launches): [1] max threads per bucket = 0, [2..3] skewed slot
// range = empty
__global__ void __launch_bounds__(1024)
    k_sort_chunks(const uint32_t* __restrict__ goff, uint32_t nblk, int H,
                  uint32_t* __restrict__ gstart, uint32_t* __restrict__ cbase,
                  uint32_t* __restrict__ chunk_group, uint32_t* __restrict__ misc) {
  __shared__ uint32_t sh[1024];
  const int g = threadIdx.x;
  if (threadIdx.x >= 1 && threadIdx.x <= 3) misc[threadIdx.x] = threadIdx.x == 2 ? 0xffffffffu : 0u;
  const uint32_t total = goff[(size_t)H * nblk];
  uint32_t gs = 0, ge = 0, nch = 0;
  if (g < H) {
    gs = goff[(size_t)g * nblk];
    ge = (g + 1 < H) ? goff[(size_t)(g + 1) * nblk] : total;
    nch = (ge - gs + SORT_CHUNK - 1) / SORT_CHUNK;
    gstart[g] = gs;
  }
  sh[threadIdx.x] = nch;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    uint32_t add = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : 0u;
    __syncthreads();
    sh[threadIdx.x] += add;
    __syncthreads();
  }
  const uint32_t cb = sh[threadIdx.x] - nch;
  if (g < H) {
    cbase[g] = cb;
    for (uint32_t k = 0; k < nch; k++) chunk_group[cb + k] = (uint32_t)g;
  }
  if (threadIdx.x == 1023) {
    gstart[H] = total;
    cbase[H] = sh[1023];
    misc[0] = sh[1023];
  }
}

__global__ void __launch_bounds__(SORT_BLOCK)
    k_sortB_hist(const uint16_t* __restrict__ tmp_l, const uint32_t* __restrict__ gstart,
                 const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ chunk_group,
                 const uint32_t* __restrict__ nchunks, int NL, uint32_t* __restrict__ chist) {
  extern __shared__ uint32_t hist[];
  const uint32_t nch = *nchunks;
  if (blockIdx.x >= nch) return;
  const uint32_t k = xcd_tile(blockIdx.x, nch);
  const uint32_t g = chunk_group[k];
  const uint32_t s = gstart[g] + (k - cbase[g]) * SORT_CHUNK;
  const uint32_t e = min(s + SORT_CHUNK, gstart[g + 1]);
  for (int l = threadIdx.x; l < NL; l += blockDim.x) hist[l] = 0;
  __syncthreads();
  constexpr int PER = SORT_CHUNK / SORT_BLOCK;
  uint32_t lv[PER];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const uint32_t p = s + threadIdx.x + j * SORT_BLOCK;
    lv[j] = p < e ? (uint32_t)tmp_l[p] : 0xffffffffu;
  }
#pragma unroll
  for (int j = 0; j < PER; j++)
    if (lv[j] != 0xffffffffu) atomicAdd(&hist[lv[j]], 1u);
  __syncthreads();
  for (int l = threadIdx.x; l < NL; l += blockDim.x) chist[(size_t)k * NL + l] = hist[l];
}

// per bucket b = (g, l): total count over the group's chunks
__global__ void k_sort_bucket_count(const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ chist,
                                    int LO, uint32_t nb, uint32_t* __restrict__ counts) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint32_t g = b >> LO, l = b & ((1u << LO) - 1);
  uint32_t c = 0;
#pragma unroll 8
  for (uint32_t k = cbase[g]; k < cbase[g + 1]; k++) c += chist[((size_t)k << LO) + l];
  counts[b] = c;
}

__global__ void k_sort_chunk_offsets(const uint32_t* __restrict__ cbase,
                                     const uint32_t* __restrict__ chist, int LO, uint32_t nb,
                                     const uint32_t* __restrict__ bstart,
                                     uint32_t* __restrict__ coff) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= nb) return;
  const uint32_t g = b >> LO, l = b & ((1u << LO) - 1);
  uint32_t run = bstart[b];
#pragma unroll 8
  for (uint32_t k = cbase[g]; k < cbase[g + 1]; k++) {
    const size_t idx = ((size_t)k << LO) + l;
    coff[idx] = run;  // chunk k's output offset for bucket b
    run += chist[idx];
  }
}

// Pass B scatter: the chunk is counting-sorted by the low bucket bits in LDS,
// then each bucket run is written contiguously at its chunk offset.
static_assert(SORT_CHUNK % SORT_BLOCK == 0, "pass-B chunk must split evenly over the block");
__global__ void __launch_bounds__(SORT_BLOCK)
    k_sortB_scatter(const uint32_t* __restrict__ tmp_e, const uint16_t* __restrict__ tmp_l,
                    const uint32_t* __restrict__ gstart,
                    const uint32_t* __restrict__ cbase, const uint32_t* __restrict__ chunk_group,
                    const uint32_t* __restrict__ nchunks, int NL, const uint32_t* __restrict__ chist,
                    const uint32_t* __restrict__ coff, uint32_t* __restrict__ entries) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t* e32 = reinterpret_cast<uint32_t*>(smem);
  uint16_t* bins = reinterpret_cast<uint16_t*>(e32 + SORT_CHUNK);
  uint32_t* loff = reinterpret_cast<uint32_t*>(bins + SORT_CHUNK);
  uint32_t* cur = loff + NL;
  uint32_t* cb = cur + NL;
  uint32_t* scr = cb + NL;
  const uint32_t nch = *nchunks;
  if (blockIdx.x >= nch) return;
  const uint32_t k = xcd_tile(blockIdx.x, nch);
  const uint32_t g = chunk_group[k];
  const uint32_t s = gstart[g] + (k - cbase[g]) * SORT_CHUNK;
  const uint32_t e = min(s + SORT_CHUNK, gstart[g + 1]);
  // all of the thread's entries are loaded first: their round trip overlaps
  // the histogram row, its scan and the offset row instead of following them
  constexpr int PER = SORT_CHUNK / SORT_BLOCK;
  uint32_t ev[PER], lv[PER];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    const uint32_t p = s + threadIdx.x + j * SORT_BLOCK;
    lv[j] = p < e ? (uint32_t)tmp_l[p] : 0xffffffffu;
    ev[j] = p < e ? tmp_e[p] : 0u;
  }
  // the chunk's histogram was computed by k_sortB_hist (chist)
  for (int l = threadIdx.x; l < NL; l += blockDim.x) {
    loff[l] = chist[(size_t)k * NL + l];
    cur[l] = 0;
  }
  __syncthreads();
  lds_exscan(loff, NL, scr);
  for (int l = threadIdx.x; l < NL; l += blockDim.x) cb[l] = coff[(size_t)k * NL + l] - loff[l];
#pragma unroll
  for (int j = 0; j < PER; j++) {
    if (lv[j] == 0xffffffffu) continue;
    const uint32_t l = lv[j];
    const uint32_t slot = loff[l] + atomicAdd(&cur[l], 1u);
    e32[slot] = ev[j];
    bins[slot] = (uint16_t)l;
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < e - s; q += blockDim.x) entries[cb[bins[q]] + q] = e32[q];
}

// ---- generic exclusive scan of uint32 (out[n] = total) -------------------
__global__ void k_scan32_tiles(const uint32_t* __restrict__ in, size_t n, uint32_t* __restrict__ out,
                               uint32_t* __restrict__ tile_tot) {
  __shared__ uint32_t sh[256];
  const size_t base = ((size_t)blockIdx.x * 256 + threadIdx.x) * 8;
  uint32_t v[8], tot = 0;
  for (int k = 0; k < 8; k++) {
    v[k] = base + k < n ? in[base + k] : 0u;
    tot += v[k];
  }
  sh[threadIdx.x] = tot;
  __syncthreads();
  for (int off = 1; off < 256; off <<= 1) {
    uint32_t add = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : 0u;
    __syncthreads();
    sh[threadIdx.x] += add;
    __syncthreads();
  }
  uint32_t run = sh[threadIdx.x] - tot;
  for (int k = 0; k < 8; k++) {
    if (base + k < n) out[base + k] = run;
    run += v[k];
  }
  if (threadIdx.x == 255) tile_tot[blockIdx.x] = sh[255];
}

__global__ void __launch_bounds__(1024)
    k_scan32_top(uint32_t* __restrict__ tile_tot, int ntiles, uint32_t* __restrict__ out_total) {
  __shared__ uint32_t sh[1024];
  const int per = (ntiles + 1023) / 1024;
  const int base = threadIdx.x * per;
  uint32_t tot = 0;
  for (int k = 0; k < per; k++)
    if (base + k < ntiles) tot += tile_tot[base + k];
  sh[threadIdx.x] = tot;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    uint32_t add = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : 0u;
    __syncthreads();
    sh[threadIdx.x] += add;
    __syncthreads();
  }
  uint32_t run = sh[threadIdx.x] - tot;
  for (int k = 0; k < per; k++) {
    if (base + k < ntiles) {
      uint32_t t = tile_tot[base + k];
      tile_tot[base + k] = run;
      run += t;
    }
  }
  if (threadIdx.x == 1023) *out_total = sh[1023];
}

__global__ void k_scan32_add(const uint32_t* __restrict__ tile_off, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += tile_off[i / 2048];
}

// ---- exclusive scan of (count, ceil(count/E)) over nb buckets -------------
static constexpr int SCAN_PER_THREAD = 8;
static constexpr int SCAN_BLOCK = 256;
static constexpr int SCAN_TILE = SCAN_PER_THREAD * SCAN_BLOCK;

// entries per accumulation thread = L (chosen per call, msm_accumulate_phase)
__device__ __forceinline__ uint2 scan_val(const uint32_t* counts, size_t i, size_t nb, uint32_t L) {
  uint32_t c = i < nb ? counts[i] : 0u;
  return make_uint2(c, (c + L - 1) / L);
}

// per-tile exclusive scan; writes tile totals
__global__ void k_scan_tiles(const uint32_t* __restrict__ counts, size_t nb, uint32_t L,
                             uint32_t* __restrict__ bstart, uint2* __restrict__ tile_tot,
                             uint32_t* __restrict__ max_tpb) {
  __shared__ uint2 sh[SCAN_BLOCK];
  size_t base = (size_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER_THREAD;
  uint2 v[SCAN_PER_THREAD];
  uint2 tot = make_uint2(0, 0);
  uint32_t mx = 0;
  for (int k = 0; k < SCAN_PER_THREAD; k++) {
    v[k] = scan_val(counts, base + k, nb, L);
    tot.x += v[k].x;
    tot.y += v[k].y;
    mx = max(mx, v[k].y);
  }
  if (mx > 1) atomicMax(max_tpb, mx);
  sh[threadIdx.x] = tot;
  __syncthreads();
  // Hillis-Steele inclusive scan of thread totals
  for (int off = 1; off < SCAN_BLOCK; off <<= 1) {
    uint2 add = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : make_uint2(0, 0);
    __syncthreads();
    sh[threadIdx.x].x += add.x;
    sh[threadIdx.x].y += add.y;
    __syncthreads();
  }
  uint2 run = threadIdx.x ? sh[threadIdx.x - 1] : make_uint2(0, 0);
  for (int k = 0; k < SCAN_PER_THREAD; k++) {
    size_t i = base + k;
    if (i < nb) bstart[i] = run.x;
    run.x += v[k].x;
    run.y += v[k].y;
  }
  if (threadIdx.x == SCAN_BLOCK - 1) tile_tot[blockIdx.x] = sh[SCAN_BLOCK - 1];
}

// single block: exclusive scan of tile totals (ntiles <= 1024 * 8)
__global__ void k_scan_top(uint2* __restrict__ tile_tot, int ntiles, uint32_t* __restrict__ bstart,
                           size_t nb) {
  __shared__ uint2 sh[1024];
  const int per = (ntiles + 1023) / 1024;
  int base = threadIdx.x * per;
  uint2 tot = make_uint2(0, 0);
  for (int k = 0; k < per; k++) {
    if (base + k < ntiles) {
      tot.x += tile_tot[base + k].x;
      tot.y += tile_tot[base + k].y;
    }
  }
  sh[threadIdx.x] = tot;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    uint2 add = threadIdx.x >= (unsigned)off ? sh[threadIdx.x - off] : make_uint2(0, 0);
    __syncthreads();
    sh[threadIdx.x].x += add.x;
    sh[threadIdx.x].y += add.y;
    __syncthreads();
  }
  uint2 run = threadIdx.x ? sh[threadIdx.x - 1] : make_uint2(0, 0);
  for (int k = 0; k < per; k++) {
    if (base + k < ntiles) {
      uint2 t = tile_tot[base + k];
      tile_tot[base + k] = run;
      run.x += t.x;
      run.y += t.y;
    }
  }
  if (threadIdx.x == 1023) bstart[nb] = sh[1023].x;
}

// final bucket starts; misc[2] / misc[3] = first / last partial slot of the
// buckets with more than T partial slots (msm_combine_run: the reduction's
// tree steps run over that range only); also resets the owner words of the
// partial slots to ~0 (the accumulation marks the slots it writes; no fill launch)
__global__ void k_scan_add(const uint2* __restrict__ tile_off, size_t nb, uint32_t* __restrict__ bstart,
                           const uint32_t* __restrict__ counts, uint32_t L, uint32_t T,
                           uint32_t* __restrict__ misc, uint32_t gen, uint32_t* __restrict__ owner,
                           size_t nslots) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (size_t o = i; o < nslots; o += (size_t)gridDim.x * blockDim.x) owner[o] = 0xffffffffu;
  if (i >= nb) return;
  if (i == 0) misc[4] = gen;  // tag of this run's plan words (checked by the reader)
  uint2 off = tile_off[i / SCAN_TILE];
  uint32_t b = bstart[i] + off.x;
  bstart[i] = b;
  const uint32_t c = counts[i];
  if (c > (T - 1) * L) {  // may span more than T slots
    const uint32_t f = b / L + (uint32_t)i, l = (b + c - 1) / L + (uint32_t)i;
    if (l - f + 1 > T) {
      atomicMin(misc + 2, f);
      atomicMax(misc + 3, l);
    }
  }
}

// ---- accumulation ---------------------------------------------------------
// Flat chunks: the bucket-sorted entries are cut into chunks of exactly L
// entries regardless of bucket boundaries, one thread per chunk, so every lane
// of a wave runs the same trip count.  A thread whose chunk crosses a bucket
// boundary stores the finished bucket's partial sum and starts a new one.  The
// partial of (thread t, bucket b) lives in slot t + b: unique, and the slots
// of bucket b are the contiguous range [t_first(b) + b, t_last(b) + b] with
// t_first(b) = bstart[b] / L, t_last(b) = (bstart[b + 1] - 1) / L.
QG_DEV void msm_flush(X29Raw* partial, uint32_t* owner, uint32_t slot, uint32_t b, const X29& acc,
                      bool inf) {
  partial[slot] = x29_raw(inf ? x29_inf() : acc);  // finished by the reader
  owner[slot] = b;
}

// e / L for the chunk length L of a launch (any multiple of 4), by one 64-bit
// high multiply with Lm = floor((2^64 - 1) / L) + 1: exact for e < 2^32 and
// L < 2^16 (the error e (Lm - 2^64 / L) / 2^64 < 2^-32 < 1 / L).  A division
// here made k_msm_accumulate<false> spill 28 B per lane (round 6).
QG_DEV uint32_t msm_chunk_of(uint32_t e, uint64_t Lm) { return (uint32_t)__umul64hi((uint64_t)e, Lm); }

QG_DEV X29 msm_partial(const X29Raw* partial, uint32_t slot) {
  return x29_acc_finish(x29_unraw(partial[slot]));
}

// entries e .. e + 3 (those < e1); one 16-B load when aligned and in range
QG_DEV uint4 msm_entries4(const uint32_t* __restrict__ entries, uint32_t e, uint32_t e1) {
  if ((e & 3u) == 0 && e + 4 <= e1) return *reinterpret_cast<const uint4*>(entries + e);
  uint4 r = make_uint4(0, 0, 0, 0);
  if (e < e1) r.x = entries[e];
  if (e + 1 < e1) r.y = entries[e + 1];
  if (e + 2 < e1) r.z = entries[e + 2];
  if (e + 3 < e1) r.w = entries[e + 3];
  return r;
}

// at most 128 VGPRs: four waves per SIMD (the paired multiplies need ~131).
// PF: the software-pipelined form (the row of entry e + 1 gathered before the
// addition of entry e), three waves per SIMD: -1.5 % at 2^24 scalars, +3 % at
// 2^20 (profiles/r04_msm_prefetch_ab.txt), so only the largest MSMs take it.
template <bool PF>
__global__ void __launch_bounds__(MSM_BLOCK) __attribute__((amdgpu_waves_per_eu(PF ? 3 : 4)))
    k_msm_accumulate(const MsmPt* __restrict__ table, const uint32_t* __restrict__ entries,
                     const uint32_t* __restrict__ bstart, uint32_t nb, uint32_t L, uint64_t Lm,
                     X29Raw* __restrict__ partial, uint32_t* __restrict__ owner) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = bstart[nb];
  const uint64_t e0w = (uint64_t)t * L;
  if (e0w >= total) return;
  const uint32_t e0 = (uint32_t)e0w;
  const uint32_t e1 = total - e0 < L ? total : e0 + L;
  // the thread index is not kept live through the loop (it cost the
  // non-prefetching form one VGPR spilled and reloaded per addition): a flush
  // recovers it from the chunk end, t = (e1 - 1) / L (msm_chunk_of); chunks start at
  // multiples of L (>= 4), so the group phase is e & 3
  // bucket of entry e0: the largest b with bstart[b] <= e0 (b < nb)
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (bstart[mid] <= e0) lo = mid;
    else hi = mid;
  }
  uint32_t b = lo;
  uint32_t next = bstart[b + 1];
  // 29-bit-limb XYZZ accumulator (lazily reduced, curve29.h x29_acc_madd_tp);
  // rows are canonical in the R = 2^261 domain, the signed digit picks y or p - y
  X29 acc;
  bool inf = true;
  if constexpr (PF) {
  uint4 g0 = msm_entries4(entries, e0, e1);
  uint4 g1 = e0 + 4 < e1 ? msm_entries4(entries, e0 + 4, e1) : g0;
  Q29 ax, ay;
#ifndef QG_MSM_ROWMASK
#define QG_MSM_ROWMASK 0x7fffffffu  // experiment builds narrow the gathered span (timing only)
#endif
  bool pinf = msm_pt_load(table, g0.x & QG_MSM_ROWMASK, (g0.x >> 31) != 0u, ax, ay);
  for (uint32_t e = e0; e < e1; e++) {
    const uint32_t k = e & 3u;
    Q29 bx = ax, by = ay;
    bool qinf = true;
    if (e + 1 < e1) {
      const uint32_t en = k == 0 ? g0.y : k == 1 ? g0.z : k == 2 ? g0.w : g1.x;
      qinf = msm_pt_load(table, en & QG_MSM_ROWMASK, (en >> 31) != 0u, bx, by);
    }
    if (k == 3) {
      g0 = g1;
      if (e + 5 < e1) g1 = msm_entries4(entries, e + 5, e1);
    }
    if (e == next) {
      msm_flush(partial, owner, msm_chunk_of(e1 - 1, Lm) + b, b, acc, inf);
      inf = true;
      do {
        b++;
        next = bstart[b + 1];
      } while (next <= e);
    }
    if (!pinf) {
      if (inf) {
        acc.X = ax;
        acc.Y = ay;
        acc.ZZ = Q29::from_l9(F29P<FqP>::ONE);
        acc.ZZZ = acc.ZZ;
        inf = false;
      } else if (!x29_acc_madd_tp(acc, ax, ay)) {
        x29_acc_madd_exc(acc, ax, ay, &inf);
      }
    }
    ax = bx;
    ay = by;
    pinf = qinf;
  }
  msm_flush(partial, owner, msm_chunk_of(e1 - 1, Lm) + b, b, acc, inf);
  return;
  }
  // entries arrive four at a time (one 16-B load per group of four, the next
  // group in flight during the current one): a thread revisits its entry line
  // only every few microseconds, long after L2 has evicted it, so single-entry
  // loads refetched a whole 128-B line per entry (as many bytes as the rows)
  uint4 cur = msm_entries4(entries, e0, e1), nxt = cur;
  for (uint32_t e = e0; e < e1; e++) {
    const uint32_t k = e & 3u;  // wave-uniform (chunks start at multiples of 4)
    if (k == 0 && e + 4 < e1) nxt = msm_entries4(entries, e + 4, e1);
    const uint32_t ent = k == 0 ? cur.x : k == 1 ? cur.y : k == 2 ? cur.z : cur.w;
    if (k == 3) cur = nxt;
    if (e == next) {  // bucket boundary (at most a few per thread)
      msm_flush(partial, owner, msm_chunk_of(e1 - 1, Lm) + b, b, acc, inf);
      inf = true;
      do {
        b++;
        next = bstart[b + 1];
      } while (next <= e);
    }
    Q29 ax, ay;
    const bool pinf = msm_pt_load(table, ent & 0x7fffffffu, (ent >> 31) != 0u, ax, ay);
    if (pinf) continue;
    if (inf) {
      acc.X = ax;
      acc.Y = ay;
      acc.ZZ = Q29::from_l9(F29P<FqP>::ONE);
      acc.ZZZ = acc.ZZ;
      inf = false;
      continue;
    }
    if (!x29_acc_madd_tp(acc, ax, ay)) x29_acc_madd_exc(acc, ax, ay, &inf);
  }
  msm_flush(partial, owner, msm_chunk_of(e1 - 1, Lm) + b, b, acc, inf);
}

// Cooperative row gathers (COOP).  One 16-B load per lane of five per row
// (msm_pt_load) puts 320 independent row requests on the memory path per wave
// step; over a 27.9 GB table the chip then serves 1.6e10 random rows/s, about
// what the accumulate consumes (micro/gather_bench.hip: 1.58e10 rows/s with
// five 16-B loads per lane, 3.37e10 with eight lanes loading one 128-B row in
// one coalesced request; the accumulate with its gathers confined to 2 GiB ran
// 16.3 -> 14.9 ms, profiles/r05_gather_ab.txt).  Here each wave step gathers
// the wave's 64 rows with eight LDS-DMA instructions (global_load_lds_dwordx4:
// lane l of instruction k loads a 16-B word of the row of lane 8k + l/8, into a
// per-wave 8 KiB LDS image), then every lane reads its own row's five words.
// The next step's DMA is in flight during this step's addition.  Word w of
// row m sits at position w ^ (m & 7) of the row's 128 B (the swizzle rides on
// the DMA source address, the LDS image stays lane-linear): the readers of a
// ds_read_b128 spread over 8 bank groups instead of 2.
typedef __attribute__((address_space(3))) void* msm_lds_ptr;
typedef __attribute__((address_space(1))) void* msm_glb_ptr;

#if defined(__HIP_DEVICE_COMPILE__)
// the eight DMA instructions of one wave step: lane l of instruction k loads
// word (l & 7) ^ (l >> 3 & 7) of the row of lane 8k + (l >> 3) (entry `ent`,
// row bits only; 0 for a lane without a next entry)
__device__ __forceinline__ void msm_coop_issue(uint4* wbuf, const MsmPt* __restrict__ table,
                                               uint32_t lane, uint32_t ent) {
  const uint32_t pos = lane & 7u;
  const uint32_t word = pos ^ ((lane >> 3) & 7u);
  uint32_t r[8];
#pragma unroll
  for (int k = 0; k < 8; k++) r[k] = (uint32_t)__shfl((int)(ent & 0x7fffffffu), 8 * k + (int)(lane >> 3), 64);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint4* g = reinterpret_cast<const uint4*>(table + r[k]) + word;
    __builtin_amdgcn_global_load_lds((msm_glb_ptr)g, (msm_lds_ptr)(wbuf + 64 * k), 16, 0, 0);
  }
}

// this lane's row from the wave image: x, y or p - y (neg), the infinity flag
__device__ __forceinline__ bool msm_coop_read(const uint4* wbuf, uint32_t lane, bool neg, Q29& x,
                                              Q29& y) {
  const uint4* row = wbuf + 8 * lane;
  const uint32_t sw = lane & 7u;
  const uint32_t wy = neg ? 4u : 2u;
  const uint4 x0 = row[0u ^ sw], x1 = row[1u ^ sw];
  const uint4 y0 = row[wy ^ sw], y1 = row[(wy + 1u) ^ sw];
  const uint4 top = row[6u ^ sw];
  x.l[0] = x0.x; x.l[1] = x0.y; x.l[2] = x0.z; x.l[3] = x0.w;
  x.l[4] = x1.x; x.l[5] = x1.y; x.l[6] = x1.z; x.l[7] = x1.w;
  y.l[0] = y0.x; y.l[1] = y0.y; y.l[2] = y0.z; y.l[3] = y0.w;
  y.l[4] = y1.x; y.l[5] = y1.y; y.l[6] = y1.z; y.l[7] = y1.w;
  x.l[8] = top.x;
  y.l[8] = neg ? top.z : top.y;
  return (top.w & 1u) != 0u;
}
#endif

#ifndef QG_COOP_WPE
#define QG_COOP_WPE 3
#endif
__global__ void __launch_bounds__(MSM_BLOCK) __attribute__((amdgpu_waves_per_eu(QG_COOP_WPE)))
    k_msm_accumulate_coop(const MsmPt* __restrict__ table, const uint32_t* __restrict__ entries,
                          const uint32_t* __restrict__ bstart, uint32_t nb, uint32_t L, uint64_t Lm,
                          X29Raw* __restrict__ partial, uint32_t* __restrict__ owner) {
#if defined(__HIP_DEVICE_COMPILE__)
  __shared__ uint4 img[MSM_BLOCK / 64][64 * 8];
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  uint4* wbuf = img[threadIdx.x >> 6];
  const uint32_t total = bstart[nb];
  const uint64_t e0w = (uint64_t)t * L;
  // whole waves stay or leave together (the DMA steps are wave-wide); lanes
  // past the end have an empty chunk and feed row 0 to the gathers
  if (__builtin_amdgcn_readfirstlane((uint32_t)(e0w >= total))) return;
  const uint32_t e0 = e0w < total ? (uint32_t)e0w : total;
  const uint32_t e1 = total - e0 < L ? total : e0 + L;
  uint32_t b = 0, next = 0;
  if (e0 < e1) {
    uint32_t lo = 0, hi = nb;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (bstart[mid] <= e0) lo = mid;
      else hi = mid;
    }
    b = lo;
    next = bstart[b + 1];
  }
  X29 acc;
  bool inf = true;
  uint4 g0 = msm_entries4(entries, e0, e1);
  uint4 g1 = e0 + 4 < e1 ? msm_entries4(entries, e0 + 4, e1) : g0;
  msm_coop_issue(wbuf, table, lane, e0 < e1 ? g0.x : 0u);
  for (uint32_t i = 0; i < L; i++) {  // wave-uniform trip count
    const uint32_t e = e0 + i;
    const uint32_t k = i & 3u;
    const uint32_t ent = k == 0 ? g0.x : k == 1 ? g0.y : k == 2 ? g0.z : g0.w;
    const uint32_t en = k == 0 ? g0.y : k == 1 ? g0.z : k == 2 ? g0.w : g1.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this step's rows have landed
    Q29 ax, ay;
    const bool pinf = msm_coop_read(wbuf, lane, (ent >> 31) != 0u, ax, ay);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // read before the image is refilled
    if (k == 3) {
      g0 = g1;
      if (e + 5 < e1) g1 = msm_entries4(entries, e + 5, e1);
    }
    if (i + 1 < L) msm_coop_issue(wbuf, table, lane, e + 1 < e1 ? en : 0u);
    if (e >= e1) continue;
    if (e == next) {
      msm_flush(partial, owner, msm_chunk_of(e1 - 1, Lm) + b, b, acc, inf);
      inf = true;
      do {
        b++;
        next = bstart[b + 1];
      } while (next <= e);
    }
    if (pinf) continue;
    if (inf) {
      acc.X = ax;
      acc.Y = ay;
      acc.ZZ = Q29::from_l9(F29P<FqP>::ONE);
      acc.ZZZ = acc.ZZ;
      inf = false;
      continue;
    }
    if (!x29_acc_madd_tp(acc, ax, ay)) x29_acc_madd_exc(acc, ax, ay, &inf);
  }
  if (e0 < e1) msm_flush(partial, owner, msm_chunk_of(e1 - 1, Lm) + b, b, acc, inf);
#endif
}

// first / last partial slot of bucket b (nonempty)
QG_DEV uint32_t msm_slot_first(const uint32_t* bstart, uint32_t b, uint32_t L) {
  return bstart[b] / L + b;
}
QG_DEV uint32_t msm_slot_last(const uint32_t* bstart, uint32_t b, uint32_t L) {
  return (bstart[b + 1] - 1) / L + b;
}

// stride between a bucket's partial slots after the tree steps: buckets with
// more than T slots (skewed digits: the short top window, small scalars) are
// pre-summed pairwise until at most T remain, so one lane of the reduction
// never adds a long run of partials while the others wait.  T = the typical
// slot count + 1 (msm_combine_run): the tree steps touch only skewed buckets.
QG_DEV uint32_t msm_slot_stride(uint32_t nslot, uint32_t T) {
  uint32_t st = 1;
  while (nslot > T * st) st <<= 1;
  return st;
}

// Segmented pairwise tree over the partial slots of the skewed buckets: after
// the steps s = 1, 2, 4, ... slot_first(b) + k st_b holds the sum of slots
// [k st_b, (k + 1) st_b) of bucket b.  Slots no thread wrote carry owner == ~0
// and are skipped.
__global__ void __launch_bounds__(MSM_BLOCK)
    k_msm_tree_step(X29Raw* __restrict__ partial, const uint32_t* __restrict__ owner,
                    const uint32_t* __restrict__ bstart, uint32_t L, uint32_t T, uint32_t s_lo,
                    uint32_t s_end, uint32_t s, uint32_t* hv, uint32_t gen) {
  msm_handover_check(hv, 2, 2, gen, 2u);  // the partials came from the side streams
  const uint32_t i = s_lo + blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= s_end) return;
  const uint32_t b = owner[i];
  if (b == 0xffffffffu) return;
  const uint32_t f = msm_slot_first(bstart, b, L), l = msm_slot_last(bstart, b, L);
  if (l - f + 1 <= T * s) return;  // this bucket is done at this level
  const uint32_t off = i - f;
  if ((off & (2 * s - 1)) == 0 && i + s <= l)
    partial[i] = x29_raw(x29_add(msm_partial(partial, i), msm_partial(partial, i + s)));
}

// ---- reduction ------------------------------------------------------------
// sum_j (j + 1) B_j over the nb buckets of every MSM of a batch:
//  * k_msm_bsum: thread t folds buckets [t S, t S + S) from the top, each
//    bucket summed from its partial slots on the fly (no bucket array):
//    run_t = sum B_j, wsum_t = sum (j - t S + 1) B_j, so the total is
//    sum_t wsum_t + S t run_t;
//  * then groups of G lanes fold (msm_fold): for pairs (A_g, Y_g) with weight
//    factor F,  sum_g A_g + F g Y_g = sum_g A_g + F sum_{g>=1} Suf_g  (Suf =
//    suffix sums of Y over the group: a shuffle scan, then a shuffle tree),
//    emitted as A' and Y' = G F sum_g Y_g, so the next level is again
//    sum_w A'_w + w Y'_w (factor 1);
//  * k_msm_wfold repeats the fold, 16 elements per wave on quads of lanes
//    (quad-cooperative additions, below) until one element is left.
// One wave per SIMD already saturates the VALU on an XYZZ addition (micro/
// add_bench.hip: 7.9 us per addition per wave at 1, 2 and 4 waves per SIMD),
// so the reduction's cost is its addition count - and its code size: an
// inlined addition is ~47 KB of instructions, so every kernel here issues all
// of its additions from ONE call site inside a loop (operands selected per
// iteration); several inlined copies overflowed the instruction cache (the
// first version of k_msm_bsum, 301 KB, ran 2.3x slower than its count).
// 2^19 buckets: 65536 lanes (S = 8), groups of 16 -> 4096 -> 256 -> 16 -> 1.
struct MsmRed {
  const X29Raw* partial;
  const uint32_t* bstart;
  uint32_t L, T;
};
// the runs of a batch of up to MSM_RED_BYVAL MSMs travel as a kernel argument
// (no host-to-device copy queued behind the accumulation: a pageable copy can
// block the host until the stream drains); larger batches copy an array
constexpr uint32_t MSM_RED_BYVAL = 8;
struct MsmRedSet {
  MsmRed r[MSM_RED_BYVAL];
};

#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ Q29 q29_shfl_down(const Q29& a, uint32_t d, int width) {
  Q29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = __shfl_down(a.l[i], d, width);
  return r;
}
__device__ __forceinline__ X29 x29_shfl_down(const X29& p, uint32_t d, int width) {
  return {q29_shfl_down(p.X, d, width), q29_shfl_down(p.Y, d, width),
          q29_shfl_down(p.ZZ, d, width), q29_shfl_down(p.ZZZ, d, width)};
}

// ---- quad-cooperative point arithmetic (latency-bound levels) -------------
// Every lane of a quad (4 lanes) holds both operands; the field products of
// one XYZZ addition / doubling are spread over the quad in dependent stages
// and the stage results broadcast back with DPP quad permutes, so every lane
// returns the full result.  Same formulas and operand bounds as x29_add /
// x29_dbl (curve29.h): 4 product stages per addition instead of 14 products
// in a row, 3 per doubling instead of 9.  micro/add_bench.hip: 4.1 us per
// addition and 2.6 us per doubling on one wave (7.9 / 4.3 us single-lane),
// for the short chains at the top of the reduction where lanes are idle.
template <int S>
__device__ __forceinline__ Q29 q29_quad(const Q29& a) {
  Q29 r;
#pragma unroll
  for (int i = 0; i < 9; i++)
    r.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.l[i], S * 0x55, 0xf, 0xf, false);
  return r;
}

__device__ __forceinline__ Q29 q29_sel(bool c, const Q29& a, const Q29& b) {
  Q29 r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

__device__ __forceinline__ X29 x29_sel(bool c, const X29& a, const X29& b) {
  return {q29_sel(c, a.X, b.X), q29_sel(c, a.Y, b.Y), q29_sel(c, a.ZZ, b.ZZ), q29_sel(c, a.ZZZ, b.ZZZ)};
}

__device__ __forceinline__ X29 x29_add_q4(const X29& p, const X29& q) {
  if (x29_is_inf(p)) return q;
  if (x29_is_inf(q)) return p;
  const uint32_t r = threadIdx.x & 3u;
  const bool r0 = r == 0, r1 = r == 1, r2 = r == 2, odd = (r & 1u) != 0u;
  // U1 = X1 ZZ2 | U2 = X2 ZZ1 | S1 = Y1 ZZZ2 | S2 = Y2 ZZZ1;  ZZ1 ZZ2 | ZZZ1 ZZZ2
  const Q29 m0 = mul29(q29_sel(r0, p.X, q29_sel(r1, q.X, q29_sel(r2, p.Y, q.Y))),
                       q29_sel(r0, q.ZZ, q29_sel(r1, p.ZZ, q29_sel(r2, q.ZZZ, p.ZZZ))));
  const Q29 m1 = mul29(q29_sel(odd, p.ZZZ, p.ZZ), q29_sel(odd, q.ZZZ, q.ZZ));
  const Q29 U1 = q29_quad<0>(m0), U2 = q29_quad<1>(m0), S1 = q29_quad<2>(m0), S2 = q29_quad<3>(m0);
  const Q29 ZZ12 = q29_quad<0>(m1), ZZZ12 = q29_quad<1>(m1);
  const Q29 P = normfull29(sub29(U2, U1));
  const Q29 R = normfull29(sub29(S2, S1));
  if (is_zero_mod29_fast<FqP, 8>(P)) return x29_add(p, q);  // doubling / cancellation (quad-uniform)
  // PP = P^2 | RR = R^2
  const Q29 sq = sqr29(q29_sel(odd, R, P));
  const Q29 PP = q29_quad<0>(sq), RR = q29_quad<1>(sq);
  // PPP = P PP | Q = U1 PP | ZZ3 = ZZ1 ZZ2 PP
  const Q29 m3 = mul29(q29_sel(r0, P, q29_sel(r1, U1, ZZ12)), PP);
  const Q29 PPP = q29_quad<0>(m3), Q = q29_quad<1>(m3), ZZ3 = q29_quad<2>(m3);
  const Q29 X3 = red16p29(sub29(sub29(sub29(RR, PPP), Q), Q));
  // Y3 = R (Q - X3) - S1 PPP | ZZZ3 = ZZZ1 ZZZ2 PPP (- 0 0)
  const Q29 z = Q29::zero();
  const Q29 m4 = red6p29(mulsub29(q29_sel(r0, R, ZZZ12), q29_sel(r0, norm29(sub29(Q, X3)), PPP),
                                  q29_sel(r0, S1, z), q29_sel(r0, PPP, z)));
  return {X3, q29_quad<0>(m4), ZZ3, q29_quad<1>(m4)};
}

__device__ __forceinline__ X29 x29_dbl_q4(const X29& p) {
  if (x29_is_inf(p)) return p;
  const uint32_t r = threadIdx.x & 3u;
  const bool r0 = r == 0, r1 = r == 1, r2 = r == 2;
  const Q29 U = normfull29(add29(p.Y, p.Y));
  // V = U^2 | X2 = X^2
  const Q29 s1 = sqr29(q29_sel((r & 1u) != 0u, p.X, U));
  const Q29 V = q29_quad<0>(s1), X2 = q29_quad<1>(s1);
  const Q29 M = normfull29(add29(add29(X2, X2), X2));
  // W = U V | S = X V | ZZ3 = ZZ V | M^2
  const Q29 m2 = mul29(q29_sel(r0, U, q29_sel(r1, p.X, q29_sel(r2, p.ZZ, M))), q29_sel(r < 3, V, M));
  const Q29 W = q29_quad<0>(m2), S = q29_quad<1>(m2), ZZ3 = q29_quad<2>(m2), MM = q29_quad<3>(m2);
  const Q29 X3 = red16p29(sub29(sub29(MM, S), S));
  // Y3 = M (S - X3) - W Y | ZZZ3 = W ZZZ (- 0 0)
  const Q29 z = Q29::zero();
  const Q29 m3 = red6p29(mulsub29(q29_sel(r0, M, W), q29_sel(r0, norm29(sub29(S, X3)), p.ZZZ),
                                  q29_sel(r0, W, z), q29_sel(r0, p.Y, z)));
  return {X3, q29_quad<0>(m3), ZZ3, q29_quad<1>(m3)};
}

template <bool Q4>
__device__ __forceinline__ X29 red_add(const X29& a, const X29& b) {
  if constexpr (Q4) return x29_add_q4(a, b);
  else return x29_add(a, b);
}
template <bool Q4>
__device__ __forceinline__ X29 red_dbl(const X29& a) {
  if constexpr (Q4) return x29_dbl_q4(a);
  else return x29_dbl(a);
}

// Group fold: element g (< mv <= 2^gl, on lane stride ES = 4 for quads, 1
// otherwise) holds (A_g, Y_g); elements >= mv hold infinity.  Afterwards
// element 0 holds A = sum_g A_g + 2^flog sum_g g Y_g and Yw = 2^ylog sum_g Y_g.
// mv is uniform over the wave; one addition and one doubling call site.
template <bool Q4>
__device__ __forceinline__ void msm_fold(X29& A, X29 Y, int gl, uint32_t mv, int flog, int ylog,
                                         X29& Yw) {
  constexpr uint32_t ES = Q4 ? 4 : 1;
  const int width = (int)(ES << gl);
  const uint32_t g = ((threadIdx.x & 63u) % (uint32_t)width) / ES;
  int ns = 0;
  while ((1u << ns) < mv) ns++;  // scan / tree steps
  X29 Yd = Y;
  for (int s = 0; s < 2 * ns + 1; s++) {
    if (s == ns) {  // suffix sums done: the doublings (one site)
      Yw = Y;
      Yd = Y;
      X29 t = Y;
      const int nd = flog > ylog ? flog : ylog;
      for (int i = 1; i <= nd; i++) {
        t = red_dbl<Q4>(t);
        if (i == flog) Yd = t;
        if (i == ylog) Yw = t;
      }
    }
    uint32_t d;
    bool live;
    X29 a, o;
    if (s < ns) {  // inclusive suffix sums of Y
      d = 1u << s;
      o = x29_shfl_down(Y, d * ES, width);
      a = Y;
      live = g + d < mv;
    } else if (s == ns) {  // + sum_{g>=1} Suf_g = sum_g g Y_g
      o = Yd;
      a = A;
      live = g != 0 && g < mv;
    } else {  // tree sum of A
      d = (1u << ns) >> (s - ns);
      o = x29_shfl_down(A, d * ES, width);
      a = A;
      live = g < d;
    }
    const X29 r = red_add<Q4>(a, x29_sel(live, o, x29_inf()));
    if (s < ns) Y = r;
    else A = r;
  }
}
#endif

// level 1 (grid.y = MSM of the batch): fold group w (2^gl lanes) writes
// A_out[w], Y_out[w] with sum_j (j + 1) B_j = sum_w A_w + w Y_w
__global__ void __launch_bounds__(MSM_BLOCK)
    k_msm_bsum(const MsmRed* __restrict__ runs, MsmRedSet rs, uint32_t nb, int slog, int gl,
               G1Xyzz* __restrict__ A_out, G1Xyzz* __restrict__ Y_out, size_t ostride,
               uint32_t* hv, uint32_t gen) {
#if defined(__HIP_DEVICE_COMPILE__)
  msm_handover_check(hv, 2, 2, gen, 2u);  // the partials came from the side streams
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const MsmRed rr = runs ? runs[blockIdx.y] : rs.r[blockIdx.y];  // small batches by value
  X29 run = x29_inf(), wsum = x29_inf(), B = x29_inf();
  const uint64_t lo64 = (uint64_t)t << slog;
  const uint32_t lo = lo64 < nb ? (uint32_t)lo64 : nb;
  uint32_t j = nb - lo < (1u << slog) ? nb : lo + (1u << slog);
  // one addition per iteration: stage 1 = bucket j += next partial slot,
  // 2 = run += B_j, 3 = wsum += run; stage 0 starts the next bucket down
  int stage = 0;
  uint32_t slot = 0, last = 0, step = 1;
  for (;;) {
    if (stage == 0) {
      if (j == lo) break;
      j--;
      const uint32_t s0 = rr.bstart[j], s1 = rr.bstart[j + 1];
      if (s0 == s1) {
        B = x29_inf();
        stage = 2;
      } else {
        const uint32_t f = s0 / rr.L + j;
        last = (s1 - 1) / rr.L + j;
        B = msm_partial(rr.partial, f);
        step = msm_slot_stride(last - f + 1, rr.T);
        slot = f + step;
        stage = slot <= last ? 1 : 2;
      }
    }
    X29 a, b;
    if (stage == 1) {
      a = B;
      b = msm_partial(rr.partial, slot);
    } else {
      a = stage == 2 ? run : wsum;
      b = stage == 2 ? B : run;
    }
    const X29 r = x29_add(a, b);
    if (stage == 1) {
      B = r;
      slot += step;
      if (slot > last) stage = 2;
    } else if (stage == 2) {
      run = r;
      stage = 3;
    } else {
      wsum = r;
      stage = 0;
    }
  }
  X29 Yw;
  msm_fold<false>(wsum, run, gl, 1u << gl, slog, gl + slog, Yw);
  if ((t & ((1u << gl) - 1)) == 0) {
    const size_t w = (size_t)blockIdx.y * ostride + (t >> gl);
    A_out[w] = x29_store(wsum);
    Y_out[w] = x29_store(Yw);
  }
#endif
}

// R = 2^261 XYZZ -> R = 2^256 Montgomery XYZZ (canonical), the host's form
QG_DEV G1Xyzz x29_export_xyzz(const X29& p) {
  if (x29_is_inf(p)) return G1Xyzz::infinity();
  return {q29_export(p.X), q29_export(p.Y), q29_export(p.ZZ), q29_export(p.ZZZ)};
}

// next levels: m elements (A_e, Y_e), total sum_e A_e + e Y_e; group w (16
// elements on quads, or 64 single-lane elements) writes (A'_w, Y'_w) of the
// same form, or only A'_w (the total) when Y_out is null, then in the host's
// form (x29_export_xyzz: the last level, no separate export launch)
template <bool Q4>
__global__ void __launch_bounds__(64)
    k_msm_wfold(const G1Xyzz* __restrict__ A_in, const G1Xyzz* __restrict__ Y_in, uint32_t m,
                size_t istride, G1Xyzz* __restrict__ A_out, G1Xyzz* __restrict__ Y_out,
                size_t ostride) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr uint32_t ES = Q4 ? 4 : 1, G = 64 / ES;
  const uint32_t e0 = blockIdx.x * G, e = e0 + threadIdx.x / ES;
  const uint32_t mv = m - e0 < G ? m - e0 : G;
  X29 A = x29_inf(), Y = x29_inf();
  if (e < m) {
    A = x29_load(A_in[(size_t)blockIdx.y * istride + e]);
    Y = x29_load(Y_in[(size_t)blockIdx.y * istride + e]);
  }
  const int gl = Q4 ? 4 : 6;
  X29 Yw;
  msm_fold<Q4>(A, Y, gl, mv, 0, Y_out ? gl : 0, Yw);
  if (threadIdx.x == 0) {
    const size_t w = (size_t)blockIdx.y * ostride + blockIdx.x;
    if (Y_out) {
      A_out[w] = x29_store(A);
      Y_out[w] = x29_store(Yw);
    } else {
      A_out[w] = x29_export_xyzz(A);
    }
  }
#endif
}

// arkworks affine points (R = 2^256 words, (0,0) = infinity) -> table rows
// (R = 2^261 canonical 29-bit limbs, y and p - y)
__global__ void k_srs_pack(const G1Affine* __restrict__ pts, size_t n, MsmPt* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const G1Affine w = pts[i];
  out[i] = w.is_inf() ? msm_pt_pack(Q29::zero(), Q29::zero(), true)
                      : msm_pt_pack(q29_import(w.x), q29_import(w.y), false);
}

// table rows -> arkworks affine points (R = 2^256 words, canonical)
__global__ void k_srs_unpack(const MsmPt* __restrict__ rows, size_t n, G1Affine* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Q29 x, y;
  if (msm_pt_unpack(rows[i], x, y)) {
    out[i] = G1Affine::infinity();
    return;
  }
  out[i] = {q29_export(x), q29_export(y)};
}

// table[w] = 2^c table[w - 1] (c doublings, one inversion back to affine)
__global__ void k_srs_shift(MsmPt* table, size_t N, int w, int c) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  A29 a;
  if (msm_pt_unpack(table[(size_t)(w - 1) * N + i], a.x, a.y)) {
    table[(size_t)w * N + i] = msm_pt_pack(Q29::zero(), Q29::zero(), true);
    return;
  }
  X29 p = x29_from_affine(a);
  for (int k = 0; k < c; k++) p = x29_dbl(p);
  // affine: x = X / ZZ, y = Y / ZZZ with one inversion
  const Q29 t = inv29(mul29(p.ZZ, p.ZZZ));
  const Q29 zzinv = mul29(t, p.ZZZ), zzzinv = mul29(t, p.ZZ);
  table[(size_t)w * N + i] = msm_pt_pack(canon29(mul29(p.X, zzinv)), canon29(mul29(p.Y, zzzinv)),
                                         false);
}

__global__ void k_powers(Fr tau, uint64_t offset, size_t n, int K, Fr* out) {
  size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t i0 = t * (size_t)K;
  if (i0 >= n) return;
  Fr x = fpow_small(tau, offset + (uint64_t)i0);
  for (int j = 0; j < K && i0 + j < n; j++) {
    out[i0 + j] = x;
    x = x * tau;
  }
}

// fixed-base comb table for g: fb[k*256 + j] = j * 2^(8k) * g, k < 32
__global__ void k_fb_powers(G1Affine g, G1Xyzz* bases) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  G1Xyzz p = G1Xyzz::from_affine(g);
  for (int k = 0; k < 32; k++) {
    bases[k] = p;
    for (int d = 0; d < 8; d++) p = xyzz_dbl(p);
  }
}

__global__ void k_fb_table(const G1Xyzz* __restrict__ bases, G1Affine* __restrict__ fb) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 32 * 256) return;
  int k = idx >> 8, j = idx & 255;
  G1Xyzz acc = xyzz_mul_small(bases[k], (uint32_t)j);
  fb[idx] = xyzz_to_affine(acc);
}

__global__ void k_fb_mul(const G1Affine* __restrict__ fb, const Fr* __restrict__ scal, size_t n,
                         G1Affine* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr s = from_mont(scal[i]);
  G1Xyzz acc = G1Xyzz::infinity();
  for (int k = 0; k < 32; k++) {
    uint32_t byte = (s.v[k >> 2] >> (8 * (k & 3))) & 255u;
    if (byte) acc = xyzz_add_affine(acc, fb[k * 256 + byte]);
  }
  out[i] = xyzz_to_affine(acc);
}

__global__ void k_import_bases(const uint64_t* __restrict__ xy, const uint8_t* __restrict__ inf,
                               size_t n, G1Affine* __restrict__ out) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  G1Affine a;
  for (int l = 0; l < 4; l++) {
    uint64_t x = xy[8 * i + l], y = xy[8 * i + 4 + l];
    a.x.v[2 * l] = (uint32_t)x;
    a.x.v[2 * l + 1] = (uint32_t)(x >> 32);
    a.y.v[2 * l] = (uint32_t)y;
    a.y.v[2 * l + 1] = (uint32_t)(y >> 32);
  }
  if (inf && inf[i]) a = G1Affine::infinity();
  out[i] = a;
}

// table 0 arrives as arkworks affine points (R = 2^256) in `base`; every row
// is kept in the R = 2^261 domain of the 29-bit-limb accumulation (curve29.h)
static void srs_build_tables(qg_ctx* ctx, qg_srs* srs, const G1Affine* base) {
  QgTimed tm(ctx, "srs_shift");
  hipLaunchKernelGGL(k_srs_pack, dim3(div_up(srs->n, 256)), dim3(256), 0, ctx->stream, base,
                     srs->n, srs->d_table);
  QG_LAUNCH_CHECK();
  for (int w = 1; w < srs->tables; w++) {
    hipLaunchKernelGGL(k_srs_shift, dim3(div_up(srs->n, 256)), dim3(256), 0, ctx->stream,
                       srs->d_table, srs->n, w, srs->c);
    QG_LAUNCH_CHECK();
  }
}

static qg_srs* srs_alloc(qg_ctx* ctx, size_t n, bool oneshot = false) {
  qg_srs* srs = new qg_srs();
  srs->ctx = ctx;
  srs->n = n;
  // balanced signed windows: W = ceil(255 / c_target), c = ceil(255 / W), so the
  // top window is not a sliver that funnels every scalar into a few buckets
  int ct = msm_window_bits(n);
  // one-shot bases: every window is a bucket set of its own in the reduction
  // (W x 2^(c-1) buckets), so the best c is smaller: 2^24 one-shot MSM 29.3 /
  // 29.6 / 30.2 / 27.9 / 28.2 / 31.0 ms at c = 20 / 20 / 19 / 18 / 17 / 16
  // (profiles/r06n_oneshot_c_sweep.txt)
  if (oneshot) ct = std::min(ct, 18);
  if (const char* ov = getenv("QG_MSM_WINDOW_BITS")) ct = atoi(ov);  // tuning experiments
  QG_CHECK(ct >= 4 && ct <= 26, QG_ERR_INVALID, "MSM window bits out of range");
  srs->W = (255 + ct - 1) / ct;
  srs->c = (255 + srs->W - 1) / srs->W;
  srs->tables = oneshot ? 1 : srs->W;
  hipError_t e = hipMalloc(&srs->d_table, (size_t)srs->tables * n * sizeof(MsmPt));
  if (e != hipSuccess) {
    delete srs;
    throw Error(QG_ERR_OOM, "qg_srs: hipMalloc of the window tables failed");
  }
  return srs;
}

// One MSM of a batch after bucketing + accumulation: its partial slots and
// bucket offsets (per-slot scratch, so a batch's reductions run together).
struct MsmRun {
  bool empty = true;
  uint32_t L = 1, T = 4;  // chunk length; partials per bucket the reduction adds in a row
  size_t nslots = 0;
  X29Raw* partial = nullptr;
  uint32_t* owner = nullptr;
  uint32_t* bstart = nullptr;
  uint32_t* misc = nullptr;  // [0] nchunks, [1] max accumulation threads per bucket,
                             // [2..3] skewed slot range, [4] generation tag
  // misc[1..3] copied to pinned host memory right after the bucket scan, and
  // its event: the reduction's launch plan waits for the bucketing only, so
  // its kernels are queued while the accumulation still runs
  const uint32_t* h_mx = nullptr;
  hipEvent_t ev_mx = nullptr;
  uint32_t gen = 0;  // misc[4] of this run: h_mx[3] must equal it
};
static constexpr int MSM_MAX_BATCH = 1024;

// bucketing (two-pass radix sort) + bucket accumulation of MSM `slot` of a
// batch: sum_i d_scalars[i] * base[srs_off + i]
//
// bst: the stream this MSM runs on.  ctx->stream (default): everything in
// stream order.  A side stream (msm_device_batch, QG_MSM_PIPE=1): the caller
// has made bst wait for the scalars; bucketing and accumulation both queue on
// bst, with their own copies of the shared bucketing scratch and entry list,
// so the next MSM's bucketing - memory-bound radix passes - runs on the other
// side stream beside this accumulation (VALU-bound, leaving a wave slot and
// LDS per CU free), and every MSM's data flows within one queue.
// reserve: only size the shared bucketing scratch and the entry list (of the
// stream `slot` selects) for an MSM of length n, launching nothing.  A batch
// reserves for its longest MSM first: a slot that grew in the middle of a
// batch would be freed while an earlier MSM's kernels still read it.
// wsel >= 0: the digits of window wsel only, over the one table of one-shot
// bases (msm_oneshot_local); -1: every window over the window-shifted tables
static MsmRun msm_accumulate_phase(qg_ctx* ctx, const qg_srs* srs, const Fr* d_scalars, size_t n,
                                   int slot, size_t srs_off = 0, hipStream_t bst = nullptr,
                                   bool reserve = false, uint32_t* hv = nullptr, uint32_t hgen = 0,
                                   int wsel = -1, bool canon_ready = false) {
  QG_CHECK(srs_off <= srs->n && n <= srs->n - srs_off, QG_ERR_INVALID, "MSM length exceeds the SRS");
  MsmRun run;
  const std::string sfx = "#" + std::to_string(slot);
  const bool side = bst != nullptr && bst != ctx->stream;
  if (!bst) bst = ctx->stream;
  // side mode: this MSM's bucketing AND accumulation run on bst, one of two
  // side streams by MSM parity, so each MSM's data flows within one queue;
  // the shared bucketing scratch and the entry list are per stream
  const std::string tg = side ? "@" + std::to_string(slot & 1) : std::string();
  if (n > 0) {
    const int c = srs->c, W = srs->W;
    QG_CHECK((wsel < 0) == (srs->tables == W) && wsel < W, QG_ERR_INVALID,
             "MSM window selection does not match the SRS tables");
    const int WE = wsel < 0 ? W : 1;  // digits per scalar this run bins
    const uint32_t nb = 1u << (c - 1);
    const size_t max_entries = n * (size_t)WE;
    QG_CHECK((size_t)W * srs->n < 0x80000000ull, QG_ERR_UNSUPPORTED, "SRS table index overflow");
    QG_CHECK(max_entries < 0xffffffffull, QG_ERR_UNSUPPORTED, "too many MSM entries");
    // bucket id b = (g << LO) | l
    const int BB = c - 1, LO = (BB + 1) / 2, HI = BB - LO;
    const int H = 1 << HI, NL = 1 << LO;
    // pass-A tile: as many scalars as fit their W digits (8 B each) in LDS
    uint32_t tile = SORT_TILE_MAX;
    while (tile > 64 && (size_t)tile * WE * 8 > SORT_LDS_A) tile >>= 1;
    if (const char* ov = getenv("QG_SORT_TILE")) tile = (uint32_t)atoi(ov);  // tuning experiments
    QG_CHECK(tile >= 64 && tile <= SORT_TILE_MAX && (tile & (tile - 1)) == 0, QG_ERR_INVALID,
             "QG_SORT_TILE must be a power of two in [64, 1024]");
    const uint32_t nblk = div_up(n, tile);
    const size_t nghist = (size_t)H * nblk;
    const size_t max_chunks = max_entries / SORT_CHUNK + H + 1;
    uint32_t* ghist = ctx->scratch_as<uint32_t>("msm_ghist" + tg, nghist + 1);
    uint32_t* goff = ctx->scratch_as<uint32_t>("msm_goff" + tg, nghist + 1);
    uint32_t* gtiles = ctx->scratch_as<uint32_t>("msm_gtiles" + tg, div_up(nghist, 2048) + 1);
    uint32_t* gstart = ctx->scratch_as<uint32_t>("msm_gstart" + tg, H + 1);
    uint32_t* cbase = ctx->scratch_as<uint32_t>("msm_cbase" + tg, H + 1);
    uint32_t* cgroup = ctx->scratch_as<uint32_t>("msm_cgroup" + tg, max_chunks);
    uint32_t* misc = ctx->scratch_as<uint32_t>("msm_misc" + sfx, 5);  // [0] nchunks, [1] max tpb
    uint32_t* chist = ctx->scratch_as<uint32_t>("msm_chist" + tg, max_chunks * NL);
    uint32_t* coff = ctx->scratch_as<uint32_t>("msm_coff" + tg, max_chunks * NL);
    uint32_t* tmp_e = ctx->scratch_as<uint32_t>("msm_tmp_e" + tg, max_entries + 1);
    uint16_t* tmp_l = ctx->scratch_as<uint16_t>("msm_tmp_l" + tg, max_entries + 1);
    uint32_t* hrow = ctx->scratch_as<uint32_t>("msm_hrow" + tg, nghist + 1);
    uint32_t* orow = ctx->scratch_as<uint32_t>("msm_orow" + tg, nghist + 1);
    Fr* canon = ctx->scratch_as<Fr>("msm_canon" + tg, n);
    uint32_t* counts = ctx->scratch_as<uint32_t>("msm_counts" + tg, nb);
    uint32_t* bstart = ctx->scratch_as<uint32_t>("msm_bstart" + sfx, nb + 1);
    uint32_t* entries = ctx->scratch_as<uint32_t>("msm_entries" + tg, max_entries + 1);
    if (reserve) return run;
    const int ntiles = (int)div_up(nb, SCAN_TILE);
    uint2* tile_tot = ctx->scratch_as<uint2>("msm_tiles" + tg, ntiles);
    // entries per accumulation thread (flat chunks, k_msm_accumulate): 64, or
    // 128 for the largest MSMs, fewer while that would leave < 3 waves of
    // threads per resident slot (256 CUs x 16 waves).  Measured against equal
    // splits into 1 / 2 / 3 whole waves of the chip (QG_MSM_ROUNDS, which also
    // leave fewer partials for the reduction): the accumulate loses 0.3-0.5 ms
    // at 2^24 with 1-2 waves, and 3 waves is no faster than 128 entries.
    uint32_t L;
    if (const char* ov = getenv("QG_MSM_ROUNDS")) {  // tuning experiments
      const int rounds = atoi(ov);
      QG_CHECK(rounds >= 1 && rounds <= 64, QG_ERR_INVALID, "QG_MSM_ROUNDS out of range");
      const size_t resident = (size_t)ctx->num_cus() * 16 * 64;
      L = 4;  // a power of two (k_msm_accumulate takes log2 L), rounded up
      while ((size_t)L * resident * rounds < max_entries) L <<= 1;
    } else {
      int elog = max_entries >= ((size_t)1 << 27) ? 7 : 6;
      while (elog > 2 && (max_entries >> elog) < (size_t)ctx->num_cus() * 16 * 64 * 3) elog--;
      // but at most ~4 chunks per bucket: below that the reduction's slot
      // merges cost more than the accumulation gains from the extra threads
      // (own-SRS MSMs, profiles/r04_msm_small_elog.txt: 2^20 / 2^18 / 2^16 at
      // c = 17 / 16 / 15 take 1.73 / 1.09 / 0.73 ms with the thread rule alone,
      // 1.69 / 0.87 / 0.69 ms with 64 / 32 / 32 entries per chunk)
      // In a batch on the side streams (HyperPlonk's openings: 2^20-2^23-scalar
      // MSMs on the c = 20 tables, many buckets per MSM) at most ~2 chunks per
      // bucket: fewer partial slots to merge, HyperPlonk reduce 73.5 / 73.9 ->
      // 63.5 / 63.3 ms per proof, proof 879.7 / 878.3 -> 872.0 / 871.7 ms
      // (profiles/r06e_msm_cpb_ab.txt); a lone MSM keeps 4 (the 2^24 headline
      // measured no better with 2).  QG_MSM_CPB overrides (A/B runs).
      int emin = 0;
      size_t cpb = side ? 2 : 4;
      if (const char* ov = getenv("QG_MSM_CPB")) cpb = (size_t)std::max(1, atoi(ov));
      while (emin < 7 && ((size_t)1 << emin) * cpb * nb < max_entries) emin++;
      elog = std::max(elog, emin);
      L = 1u << elog;
    }
    if (const char* ov = getenv("QG_MSM_ELOG")) L = 1u << atoi(ov);  // tuning experiments
    // the accumulate form (below) and its resident waves per SIMD
    bool pf = max_entries >= ((size_t)1 << 27);
    if (const char* ov = getenv("QG_MSM_PF")) pf = atoi(ov) != 0;
    bool coop = max_entries >= ((size_t)1 << 25);
    if (const char* ov = getenv("QG_MSM_COOP")) coop = atoi(ov) != 0;
    // Equal chunks (any multiple of 4 entries) filling exactly k rounds of the
    // chip's resident waves: no partly-filled last round, and fewer, longer
    // chunks leave fewer partial slots per bucket for the reduction.  The MSMs
    // of a side-stream batch take k = 1: HyperPlonk 866.9 / 870.6 -> 847.1 /
    // 850.5 ms per proof, its reduce 63.3 -> 52.1 ms (the accumulate itself
    // slower, the other stream's bucketing beside it faster), 2^24 headline
    // unchanged (profiles/r06g_msm_eqsplit_ab.txt).  A lone MSM keeps the
    // power-of-two rule: with k = 1 / 2 / 3 the 2^24 accumulate is 1.4 / 0.7 /
    // 0.5 ms slower for a reduction 0.20 / 0.10 / 0.18 ms faster (the waves of
    // one round do not finish together; many rounds even them out).
    // QG_MSM_EQSPLIT=k overrides (0: the power-of-two rule; A/B runs).
    int eqk = side ? 1 : 0;
    if (const char* ov = getenv("QG_MSM_EQSPLIT")) eqk = atoi(ov);
    {
      const int k = eqk;
      if (k > 0) {
        const size_t wpe = coop ? QG_COOP_WPE : (pf ? 3 : 4);
        const size_t resident = (size_t)ctx->num_cus() * 4 * wpe * 64;
        const size_t lq = (div_up(max_entries, resident * (size_t)k) + 3) & ~(size_t)3;
        L = (uint32_t)std::max<size_t>(4, lq);
      }
    }
    // partial slots a bucket's sum adds in a row in the reduction: the typical
    // count + 1 (a bucket of c entries spans ceil(c / L) or one more slots);
    // skewed buckets beyond it are pre-summed by tree steps
    const uint32_t T = std::max<uint32_t>(4, (uint32_t)div_up(div_up(max_entries, nb), L) + 2);
    // k_msm_accumulate takes the group phase of entry e as e & 3: chunks start
    // at multiples of 4
    QG_CHECK(L >= 4 && L <= 65536 && (L & 3u) == 0, QG_ERR_INVALID, "MSM chunk length out of range");
    const uint64_t Lm = ~0ull / L + 1;  // msm_chunk_of's multiplier
    const size_t max_threads = div_up(max_entries, L);
    const size_t nslots = max_threads + nb + 1;  // partial slot of (thread t, bucket b): t + b
    X29Raw* partial = ctx->scratch_as<X29Raw>("msm_partial" + sfx, nslots);
    uint32_t* owner = ctx->scratch_as<uint32_t>("msm_owner" + sfx, nslots);
    QG_CHECK(ntiles <= 1024 * 64 && H <= 1024 && NL <= 4096, QG_ERR_UNSUPPORTED,
             "bucket count too large");
    QG_CHECK(nslots < 0xffffffffull && max_chunks < 0xffffffffull, QG_ERR_UNSUPPORTED,
             "MSM too large");

    {
      // on the side stream the region is the bucketing's span there, overlapped
      // with the previous MSM's accumulation: its own name
      QgTimed tm(ctx, side ? "msm_bucketing_side" : "msm_bucketing", bst);
      // pass A: partition digits by the high bucket bits
      hipLaunchKernelGGL(k_sortA_hist, dim3(nblk), dim3(SORT_BLOCK), H * sizeof(uint32_t),
                         bst, d_scalars, n, c, W, LO, H, nblk, tile, hrow, canon, hv, hgen, wsel,
                         canon_ready ? 1 : 0);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_transpose32, dim3(div_up(H, 32), div_up(nblk, 32)), dim3(256), 0,
                         bst, hrow, nblk, (uint32_t)H, ghist);
      QG_LAUNCH_CHECK();
      const unsigned gt = div_up(nghist, 2048);
      QG_CHECK(gt <= 1024u * 1024u, QG_ERR_UNSUPPORTED, "histogram too large");
      hipLaunchKernelGGL(k_scan32_tiles, dim3(gt), dim3(256), 0, bst, ghist, nghist, goff,
                         gtiles);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan32_top, dim3(1), dim3(1024), 0, bst, gtiles, (int)gt,
                         goff + nghist);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan32_add, dim3(div_up(nghist, 256)), dim3(256), 0, bst, gtiles,
                         nghist, goff);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_transpose32, dim3(div_up(nblk, 32), div_up(H, 32)), dim3(256), 0,
                         bst, goff, (uint32_t)H, nblk, orow);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_sortA_rows, dim3(nblk), dim3(SORT_BLOCK), 0, bst, hrow, orow, H);
      QG_LAUNCH_CHECK();
      const size_t smemA = (size_t)tile * WE * 8 + (3 * (size_t)H + SORT_BLOCK) * 4;
      QG_CHECK(smemA <= 160 * 1024, QG_ERR_UNSUPPORTED, "pass-A tile exceeds LDS");
      // the >64 KiB dynamic-LDS attribute, once per context (= per device and
      // per calling thread: a context is used by one thread at a time)
      if (ctx->memo.count("msm_lds_attr") == 0) {
        QG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sortA_scatter),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        QG_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_sortB_scatter),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
        ctx->memo["msm_lds_attr"] = "1";
      }
      hipLaunchKernelGGL(k_sortA_scatter, dim3(nblk), dim3(SORT_BLOCK), smemA, bst,
                         canon, n, srs->n, srs_off, c, W, LO, H, nblk, tile, hrow, orow, tmp_e, tmp_l,
                         wsel);
      QG_LAUNCH_CHECK();
      // pass B: sort every group by the low bits, in chunks
      hipLaunchKernelGGL(k_sort_chunks, dim3(1), dim3(1024), 0, bst, goff, nblk, H,
                         gstart, cbase, cgroup, misc);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_sortB_hist, dim3((unsigned)max_chunks), dim3(SORT_BLOCK),
                         NL * sizeof(uint32_t), bst, tmp_l, gstart, cbase, cgroup, misc, NL,
                         chist);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_sort_bucket_count, dim3(div_up(nb, 256)), dim3(256), 0, bst,
                         cbase, chist, LO, nb, counts);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(SCAN_BLOCK), 0, bst, counts,
                         (size_t)nb, L, bstart, tile_tot, misc + 1);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, bst, tile_tot, ntiles,
                         bstart, (size_t)nb);
      QG_LAUNCH_CHECK();
      run.gen = ++ctx->msm_gen;
      hipLaunchKernelGGL(k_scan_add, dim3(div_up(nb, 256)), dim3(256), 0, bst, tile_tot,
                         (size_t)nb, bstart, counts, L, T, misc, run.gen, owner, nslots);
      QG_LAUNCH_CHECK();
      {
        QG_CHECK(slot >= 0 && slot < MSM_MAX_BATCH, QG_ERR_UNSUPPORTED, "MSM batch too large");
        uint32_t* hmx =
            reinterpret_cast<uint32_t*>(ctx->pinned_get("msm_mx", MSM_MAX_BATCH * 4 * sizeof(uint32_t)));
        QG_HIP(hipMemcpyAsync(hmx + 4 * slot, misc + 1, 4 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                              bst));
        run.ev_mx = ctx->ev_get();
        QG_HIP(hipEventRecord(run.ev_mx, bst));
        run.h_mx = hmx + 4 * slot;
      }
      hipLaunchKernelGGL(k_sort_chunk_offsets, dim3(div_up(nb, 256)), dim3(256), 0, bst,
                         cbase, chist, LO, nb, bstart, coff);
      QG_LAUNCH_CHECK();
      const size_t smemB = (size_t)SORT_CHUNK * 6 + (3 * (size_t)NL + SORT_BLOCK) * 4;
      hipLaunchKernelGGL(k_sortB_scatter, dim3((unsigned)max_chunks), dim3(SORT_BLOCK), smemB,
                         bst, tmp_e, tmp_l, gstart, cbase, cgroup, misc, NL, chist, coff,
                         entries);
      QG_LAUNCH_CHECK();
    }
    const hipStream_t ast = bst;  // the accumulation follows on the same stream
    {
      QgTimed tm(ctx, "msm_accumulate", ast);
      // the prefetching per-lane-gather form (QG_MSM_PF=1 with QG_MSM_COOP=0;
      // the default for 2^27+ entries before the cooperative gathers)
      // (pf / coop chosen above) cooperative row gathers from 2^25 entries
      // (2^22 scalars x 13 windows): 2^24 accumulate 16.4-16.6 -> 15.3 ms, 2^22
      // -4 %, 2^20 neutral (profiles/r05_msm_coop_ab.txt); QG_MSM_COOP=0/1
      // forces it (A/B runs)
      if (coop)
        hipLaunchKernelGGL(k_msm_accumulate_coop, dim3(div_up(max_threads, MSM_BLOCK)),
                           dim3(MSM_BLOCK), 0, ast, srs->d_table, entries, bstart, nb, L, Lm,
                           partial, owner);
      else if (pf)
        hipLaunchKernelGGL(k_msm_accumulate<true>, dim3(div_up(max_threads, MSM_BLOCK)),
                           dim3(MSM_BLOCK), 0, ast, srs->d_table, entries, bstart, nb, L, Lm,
                           partial, owner);
      else
        hipLaunchKernelGGL(k_msm_accumulate<false>, dim3(div_up(max_threads, MSM_BLOCK)),
                           dim3(MSM_BLOCK), 0, ast, srs->d_table, entries, bstart, nb, L, Lm,
                           partial, owner);
      QG_LAUNCH_CHECK();
    }
    run.empty = n == 0;
    run.L = L;
    run.T = T;
    run.nslots = nslots;
    run.partial = partial;
    run.owner = owner;
    run.bstart = bstart;
    run.misc = misc;
  }
  return run;
}

// Bucket reduction of a batch of accumulated MSMs (same SRS): tree steps for
// skewed buckets (per MSM, rare), then ONE launch each of the bucket combine,
// the two weighted-sum levels and the export for the whole batch — the
// latency-bound tail of the MSM is paid once per batch.  out: XYZZ (R = 2^256)
// per MSM, not yet summed over ranks.
// hv / hgen: the hand-over guard words of a batch whose partials come from
// the side streams (msm_device_batch); its error word lands in *h_err (pinned)
// with the results
static void msm_reduce_phase(qg_ctx* ctx, const qg_srs* srs, const std::vector<MsmRun>& runs,
                             std::vector<G1Xyzz>& out, uint32_t* hv = nullptr, uint32_t hgen = 0,
                             uint32_t* h_err = nullptr) {
  const uint32_t k = (uint32_t)runs.size();
  out.assign(k, G1Xyzz::infinity());
  std::vector<uint32_t> live;
  for (uint32_t i = 0; i < k; i++)
    if (!runs[i].empty) live.push_back(i);
  if (live.empty()) {
    if (hv) {  // nothing to reduce: the guard word alone
      QG_HIP(hipMemcpyAsync(h_err, hv + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
      ctx->sync();
    }
    return;
  }
  QG_CHECK(live.size() <= (size_t)MSM_MAX_BATCH, QG_ERR_UNSUPPORTED, "MSM batch too large");
  const uint32_t kl = (uint32_t)live.size();
  const uint32_t nb = 1u << (srs->c - 1);
  // per MSM: max accumulation threads per bucket, and the partial-slot range of
  // the buckets the tree steps pre-sum, from the pinned copies queued after
  // each bucket scan (waiting on those events only: the accumulations keep
  // running while the reduction's kernels are queued behind them)
  std::vector<uint32_t> mx(3 * (size_t)kl);
  // QG_MSM_SYNC_PLAN=1: wait for the whole stream first (the round-3 timing, A/B runs)
  if (const char* ov = getenv("QG_MSM_SYNC_PLAN"))
    if (atoi(ov) != 0) QG_HIP(hipStreamSynchronize(ctx->stream));
  for (uint32_t q = 0; q < kl; q++) {
    const MsmRun& r = runs[live[q]];
    QG_CHECK(r.ev_mx && r.h_mx, QG_ERR_ASSERT, "MSM run without its bucket-scan event");
    QG_HIP(hipEventSynchronize(r.ev_mx));
    if (r.h_mx[3] == r.gen) {
      for (int i = 0; i < 3; i++) mx[3 * q + i] = r.h_mx[i];
    } else {  // the pinned copy is not this run's: read the words in stream order
      QG_HIP(hipStreamSynchronize(ctx->stream));
      uint32_t w[4];
      QG_HIP(hipMemcpy(w, r.misc + 1, sizeof(w), hipMemcpyDeviceToHost));
      QG_CHECK(w[3] == r.gen, QG_ERR_ASSERT, "MSM bucket-scan plan words of another run");
      for (int i = 0; i < 3; i++) mx[3 * q + i] = w[i];
      ctx->msm_plan_refetch++;
    }
  }
  for (const MsmRun& r : runs)
    if (r.ev_mx) ctx->event_pool.push_back(r.ev_mx);
  // level 1: S = 2^slog1 buckets per thread, as many threads as the chip has
  // SIMD lanes (one wave per SIMD) over the whole batch; folds of 2^gl1 lanes
  const size_t lanes = (size_t)ctx->num_cus() * 4 * 64;
  int slog1 = 0;
  while (slog1 < 12 && ((size_t)kl * nb >> (slog1 + 1)) >= lanes) slog1++;
  if (const char* ov = getenv("QG_MSM_SLOG1")) slog1 = atoi(ov);  // tuning experiments
  QG_CHECK(slog1 >= 0 && slog1 <= 12, QG_ERR_INVALID, "QG_MSM_SLOG1 out of range");
  int gl1 = 4;
  if (const char* ov = getenv("QG_MSM_GL1")) gl1 = atoi(ov);  // tuning experiments
  QG_CHECK(gl1 >= 0 && gl1 <= 6, QG_ERR_INVALID, "QG_MSM_GL1 out of range");
  const uint32_t g1 = div_up(div_up(nb, (size_t)1 << slog1), MSM_BLOCK);
  const uint32_t m1 = g1 * (MSM_BLOCK >> gl1);  // level-1 groups per MSM
  const uint32_t m2 = div_up(m1, 16);
  G1Xyzz* A1 = ctx->scratch_as<G1Xyzz>("msm_redA1", (size_t)kl * m1);
  G1Xyzz* Y1 = ctx->scratch_as<G1Xyzz>("msm_redY1", (size_t)kl * m1);
  G1Xyzz* A2 = ctx->scratch_as<G1Xyzz>("msm_redA2", (size_t)kl * m2);
  G1Xyzz* Y2 = ctx->scratch_as<G1Xyzz>("msm_redY2", (size_t)kl * m2);
  G1Xyzz* d_out = ctx->scratch_as<G1Xyzz>("msm_out", kl);
  std::vector<MsmRed> h_runs(kl);
  MsmRedSet rset{};
  {
    QgTimed tm(ctx, "msm_reduce");
    // tree steps only until every bucket has <= T partials left;
    // level 1 adds those sequentially.  A bucket of count c spans at most
    // ceil(c / L) + 1 slots.
    for (uint32_t q = 0; q < kl; q++) {
      const MsmRun& r = runs[live[q]];
      const uint32_t max_slots = mx[3 * q] + 1, s_lo = mx[3 * q + 1], s_hi = mx[3 * q + 2];
      uint32_t st = 1;
      while (s_lo <= s_hi && (size_t)st * r.T < max_slots) {
        QG_CHECK(s_hi < r.nslots, QG_ERR_ASSERT, "MSM partial-slot range");
        hipLaunchKernelGGL(k_msm_tree_step, dim3(div_up(s_hi - s_lo + 1, MSM_BLOCK)), dim3(MSM_BLOCK),
                           0, ctx->stream, r.partial, r.owner, r.bstart, r.L, r.T, s_lo, s_hi + 1,
                           st, hv, hgen);
        QG_LAUNCH_CHECK();
        st <<= 1;
      }
      h_runs[q] = {r.partial, r.bstart, r.L, r.T};
      if (q < MSM_RED_BYVAL) rset.r[q] = h_runs[q];
    }
    const MsmRed* d_runs = nullptr;
    if (kl > MSM_RED_BYVAL) {  // through pinned staging: a pageable copy queued behind
                               // the side streams would block the host until they drain
      MsmRed* d = ctx->scratch_as<MsmRed>("msm_runs", kl);
      MsmRed* hs = reinterpret_cast<MsmRed*>(ctx->pinned_get("msm_runs_h", MSM_MAX_BATCH * sizeof(MsmRed)));
      std::copy(h_runs.begin(), h_runs.end(), hs);
      QG_HIP(hipMemcpyAsync(d, hs, kl * sizeof(MsmRed), hipMemcpyHostToDevice, ctx->stream));
      d_runs = d;
    }
    hipLaunchKernelGGL(k_msm_bsum, dim3(g1, kl), dim3(MSM_BLOCK), 0, ctx->stream, d_runs, rset, nb,
                       slog1, gl1, A1, Y1, (size_t)m1, hv, hgen);
    QG_LAUNCH_CHECK();
    // wave folds, 64 elements per wave, until one element per MSM is left
    G1Xyzz *Ai = A1, *Yi = Y1, *Ao = A2, *Yo = Y2;
    size_t istride = m1;
    uint32_t m = m1;
    // (quad-cooperative folds of 16 by default: the lanes are idle up here)
    bool q4 = true;
    if (const char* ov = getenv("QG_MSM_Q4")) q4 = atoi(ov) != 0;  // A/B experiments
    const uint32_t per = q4 ? 16 : 64;
    auto fold = q4 ? k_msm_wfold<true> : k_msm_wfold<false>;
    while (m > per) {
      const uint32_t mo = div_up(m, per);
      hipLaunchKernelGGL(fold, dim3(mo, kl), dim3(64), 0, ctx->stream, Ai, Yi, m, istride, Ao, Yo,
                         (size_t)mo);
      QG_LAUNCH_CHECK();
      std::swap(Ai, Ao);
      std::swap(Yi, Yo);
      istride = mo;
      m = mo;
    }
    // the last fold writes the totals in the host's form
    hipLaunchKernelGGL(fold, dim3(1, kl), dim3(64), 0, ctx->stream, Ai, Yi, m, istride, d_out,
                       (G1Xyzz*)nullptr, (size_t)1);
    QG_LAUNCH_CHECK();
  }
  std::vector<G1Xyzz> h(kl);
  QG_HIP(hipMemcpyAsync(h.data(), d_out, kl * sizeof(G1Xyzz), hipMemcpyDeviceToHost, ctx->stream));
  if (hv) QG_HIP(hipMemcpyAsync(h_err, hv + 1, sizeof(uint32_t), hipMemcpyDeviceToHost, ctx->stream));
  ctx->sync();
  for (uint32_t q = 0; q < kl; q++) out[live[q]] = h[q];
}

// per-rank XYZZ partial -> the MSM over all ranks, affine (allgather + host EC
// adds: RCCL cannot add curve points)
static G1Affine msm_finish_ranks(qg_ctx* ctx, G1Xyzz acc) {
  if (ctx->sharded) {
    G1Xyzz* d_send = ctx->scratch_as<G1Xyzz>("msm_comm_send", 1);
    G1Xyzz* d_recv = ctx->scratch_as<G1Xyzz>("msm_comm_recv", ctx->world);
    QG_HIP(hipMemcpyAsync(d_send, &acc, sizeof(G1Xyzz), hipMemcpyHostToDevice, ctx->stream));
    comm_allgather_bytes(ctx, d_send, d_recv, sizeof(G1Xyzz));
    std::vector<G1Xyzz> all(ctx->world);
    QG_HIP(hipMemcpyAsync(all.data(), d_recv, sizeof(G1Xyzz) * ctx->world, hipMemcpyDeviceToHost,
                          ctx->stream));
    ctx->sync();
    acc = G1Xyzz::infinity();
    for (int r = 0; r < ctx->world; r++) acc = xyzz_add(acc, all[r]);
  }
  return xyzz_to_affine(acc);
}

// per-rank XYZZ partials of a batch -> the MSMs over all ranks, affine: one
// allgather of the k partials (a sharded batch of openings exchanges once per
// MSM batch, not once per MSM)
static std::vector<G1Affine> msm_finish_ranks_batch(qg_ctx* ctx, const std::vector<G1Xyzz>& loc) {
  const size_t k = loc.size();
  std::vector<G1Affine> res(k);
  if (!ctx->sharded || k == 0) {
    for (size_t i = 0; i < k; i++) res[i] = xyzz_to_affine(loc[i]);
    return res;
  }
  if (k == 1) {
    res[0] = msm_finish_ranks(ctx, loc[0]);
    return res;
  }
  const size_t W = (size_t)ctx->world;
  G1Xyzz* d_send = ctx->scratch_as<G1Xyzz>("msm_comm_send", k);
  G1Xyzz* d_recv = ctx->scratch_as<G1Xyzz>("msm_comm_recv", k * W);
  QG_HIP(hipMemcpyAsync(d_send, loc.data(), k * sizeof(G1Xyzz), hipMemcpyHostToDevice, ctx->stream));
  comm_allgather_bytes(ctx, d_send, d_recv, k * sizeof(G1Xyzz));
  std::vector<G1Xyzz> all(k * W);
  QG_HIP(hipMemcpyAsync(all.data(), d_recv, k * W * sizeof(G1Xyzz), hipMemcpyDeviceToHost,
                        ctx->stream));
  ctx->sync();
  for (size_t i = 0; i < k; i++) {
    G1Xyzz acc = G1Xyzz::infinity();
    for (size_t r = 0; r < W; r++) acc = xyzz_add(acc, all[r * k + i]);
    res[i] = xyzz_to_affine(acc);
  }
  return res;
}

// k MSMs over the same SRS (KZG openings of one proof); results per MSM,
// summed over the RCCL ranks when a communicator is attached
//
// Batches of two or more MSMs run on two side streams by MSM parity, each
// MSM's bucketing and accumulation on one stream: MSM i + 1's radix passes
// (memory-bound) run beside MSM i's accumulation (VALU-bound), which slows
// by ~0.3 ms per 1 ms of bucketing it hosts.  HyperPlonk proof 935.8 / 932.6
// -> 896.1 / 894.9 ms (profiles/r05_msm_pipe2_ab.txt).
//
// The two cross-stream hand-overs are event-ordered: the scalars (written on
// ctx->stream) go to both side streams behind one event, the partial sums come
// back to the reduction (ctx->stream) behind one event per side stream.  Each
// event is fresh for its hand-over and returns to the pool only after the
// batch's final synchronization, and each hand-over is checked on the device
// (the guard words above k_sortA_hist): a consumer block that starts before its
// producer stream reached the tag sets an error bit; the host then recomputes
// the batch in stream order and counts it (`msm_handover_violation`, in the
// bench line).  Round 5 had crossed these hand-overs through host
// synchronizations after intermittently wrong quotient commitments with
// event-ordered forms; micro/handover_probe.hip (profiles/r06_handover_probe.txt)
// then found no ordering or visibility failure of event hand-overs themselves
// in ~1.3e5 checked hand-overs (RAW and WAW, held and LIFO-recycled events, a
// D2H copy as the last producer command, under load), DESIGN §5.3 has the
// analysis.  QG_MSM_PIPE=0 keeps a batch on ctx->stream; QG_MSM_PIPE_SYNC=1
// crosses through host synchronizations instead of events (A/B runs).
// One-shot bases (qg_bases_upload: ONE table, no window-shifted copies): the
// W windows of an MSM are W runs over that table, run w binning only the w-th
// signed digit of every scalar into its 2^(c-1) buckets (k_sortA_* wsel); the
// runs share one batched reduction, and the window sums R_w combine as
// sum_w 2^(c w) R_w by Horner steps on the host (c doublings + one addition per
// window, ~260 XYZZ operations).  It pays W bucketing passes over the scalars
// and W bucket sets in the reduction instead of the W - 1 table shifts a fixed
// SRS pays once (k_srs_shift, 0.63 s at 2^24), so a caller of msm_unchecked
// with bases it uses once (ark-ec's VariableBaseMSM::msm_unchecked, kzg.rs:72)
// need not build 13 tables for one MSM.
static G1Xyzz msm_oneshot_local(qg_ctx* ctx, const qg_srs* srs, const Fr* d, size_t n,
                                size_t srs_off = 0) {
  if (n == 0) return G1Xyzz::infinity();
  std::vector<MsmRun> runs;
  // all on ctx->stream: window w > 0 reads the canonical scalars window 0's
  // pass A left in the (per-stream) canon scratch
  for (int w = 0; w < srs->W; w++)
    runs.push_back(
        msm_accumulate_phase(ctx, srs, d, n, w, srs_off, nullptr, false, nullptr, 0, w, w > 0));
  std::vector<G1Xyzz> part;
  msm_reduce_phase(ctx, srs, runs, part);  // ends with a synchronization
  G1Xyzz acc = part[srs->W - 1];
  for (int w = srs->W - 2; w >= 0; w--) {
    for (int k = 0; k < srs->c; k++) acc = xyzz_dbl(acc);
    acc = xyzz_add(acc, part[w]);
  }
  return acc;
}

static std::vector<G1Xyzz> msm_batch_local(qg_ctx* ctx, const qg_srs* srs,
                                           const std::vector<const Fr*>& scalars,
                                           const std::vector<size_t>& ns, bool pipe,
                                           bool* violated) {
  *violated = false;
  if (srs->tables != srs->W) {  // one-shot bases: each MSM window by window, stream order
    std::vector<G1Xyzz> local;
    for (size_t i = 0; i < scalars.size(); i++)
      local.push_back(msm_oneshot_local(ctx, srs, scalars[i], ns[i]));
    return local;
  }
  hipStream_t side[2] = {nullptr, nullptr};
  bool host_sync = false;
  if (const char* ov = getenv("QG_MSM_PIPE_SYNC")) host_sync = atoi(ov) != 0;
  std::vector<hipEvent_t> held;  // hand-over events of this batch
  uint32_t* hv = nullptr;
  uint32_t hgen = 0;
  uint32_t* h_err = nullptr;
  if (pipe) {
    if (!ctx->side_stream) QG_HIP(hipStreamCreateWithFlags(&ctx->side_stream, hipStreamNonBlocking));
    if (!ctx->side_stream2) QG_HIP(hipStreamCreateWithFlags(&ctx->side_stream2, hipStreamNonBlocking));
    side[0] = ctx->side_stream;
    side[1] = ctx->side_stream2;
    if (host_sync) {
      QG_HIP(hipStreamSynchronize(ctx->stream));
    } else {
      hv = ctx->scratch_as<uint32_t>("msm_handover", 4);
      h_err = reinterpret_cast<uint32_t*>(ctx->pinned_get("msm_handover_h", 16));
      hgen = ++ctx->msm_gen;
      hipLaunchKernelGGL(k_handover_tag, dim3(1), dim3(64), 0, ctx->stream, hv, 0u, hgen, 1u);
      QG_LAUNCH_CHECK();
      hipEvent_t ev = ctx->ev_get();
      held.push_back(ev);
      QG_HIP(hipEventRecord(ev, ctx->stream));
      for (hipStream_t st : side) QG_HIP(hipStreamWaitEvent(st, ev, 0));
    }
  }
  if (scalars.size() >= 2) {  // size the shared scratch for the longest MSM first
    size_t im = 0;
    for (size_t i = 1; i < ns.size(); i++)
      if (ns[i] > ns[im]) im = i;
    for (int p = 0; p < (pipe ? 2 : 1); p++)
      msm_accumulate_phase(ctx, srs, scalars[im], ns[im], p, 0, side[p], true);
  }
  std::vector<MsmRun> runs;
  for (size_t i = 0; i < scalars.size(); i++)
    runs.push_back(
        msm_accumulate_phase(ctx, srs, scalars[i], ns[i], (int)i, 0, side[i & 1], false, hv, hgen));
  if (pipe && host_sync) {
    for (hipStream_t st : side) QG_HIP(hipStreamSynchronize(st));
  } else if (pipe) {  // the reduction (ctx->stream) after both side streams
    for (int p = 0; p < 2; p++) {
      hipLaunchKernelGGL(k_handover_tag, dim3(1), dim3(64), 0, side[p], hv, 2u + (uint32_t)p, hgen, 0u);
      QG_LAUNCH_CHECK();
      hipEvent_t ev = ctx->ev_get();
      held.push_back(ev);
      QG_HIP(hipEventRecord(ev, side[p]));
      QG_HIP(hipStreamWaitEvent(ctx->stream, ev, 0));
    }
  }
  std::vector<G1Xyzz> local;
  // ends with a synchronization of ctx->stream, which waited for both side
  // streams: the side streams are idle when this returns (the grid-barrier
  // sumcheck kernels never share the chip with them)
  msm_reduce_phase(ctx, srs, runs, local, hv, hgen, h_err);
  for (hipEvent_t e : held) ctx->event_pool.push_back(e);
  if (hv && *h_err != 0) {
    ctx->msm_handover_violation++;
    *violated = true;
  }
  return local;
}

std::vector<G1Affine> msm_device_batch(qg_ctx* ctx, const qg_srs* srs,
                                       const std::vector<const Fr*>& scalars,
                                       const std::vector<size_t>& ns) {
  QG_CHECK(scalars.size() == ns.size(), QG_ERR_INVALID, "MSM batch shape");
  bool pipe = scalars.size() >= 2 && srs->tables == srs->W;
  if (const char* ov = getenv("QG_MSM_PIPE")) pipe = pipe && atoi(ov) != 0;
  bool violated = false;
  std::vector<G1Xyzz> local = msm_batch_local(ctx, srs, scalars, ns, pipe, &violated);
  if (violated)  // a hand-over was not ordered: the batch again, in stream order
    local = msm_batch_local(ctx, srs, scalars, ns, false, &violated);
  // QG_MSM_VERIFY_BATCH=1 (diagnosis): every side-stream batch again in stream
  // order; a differing MSM is reported on stderr (micro/handover_dbg.py)
  if (pipe && getenv("QG_MSM_VERIFY_BATCH")) {
    bool v2 = false;
    std::vector<G1Xyzz> chk = msm_batch_local(ctx, srs, scalars, ns, false, &v2);
    for (size_t i = 0; i < chk.size(); i++) {
      const G1Affine a = xyzz_to_affine(local[i]), b = xyzz_to_affine(chk[i]);
      if (memcmp(&a, &b, sizeof(a)) != 0)
        fprintf(stderr, "QG_MSM_VERIFY_BATCH: MSM %zu of %zu (n = %zu) differs from stream order\n",
                i, chk.size(), ns[i]);
    }
  }
  return msm_finish_ranks_batch(ctx, local);
}

// MSM of host-resident scalars (qg_kzg_commit / qg_msm_g1): the scalars go up
// in P pieces on a copy stream and piece k's bucketing + accumulation, queued
// before the host starts the (host-blocking, pageable) copy of piece k + 1,
// runs under that copy; the pieces share one batched reduction and their
// partial sums are added.  P = n / 2^21 pieces, at most 8 (2^24 on MI355X:
// 33.0 ms with the whole copy first, 25.8 / 23.8 / 23.5 ms in 2 / 4 / 8
// pieces; profiles/r03_host_commit_pieces.txt); QG_MSM_PIECES overrides.
static G1Affine msm_host(qg_ctx* ctx, const qg_srs* srs, const uint64_t* h, size_t n) {
  Fr* d = ctx->scratch_as<Fr>("msm_scalars", n ? n : 1);
  int P = (int)std::min<size_t>(8, std::max<size_t>(1, n >> 21));
  if (const char* ov = getenv("QG_MSM_PIECES")) P = atoi(ov);  // tuning experiments
  QG_CHECK(P >= 1 && P <= 64, QG_ERR_INVALID, "QG_MSM_PIECES out of range");
  if (P == 1 || n < (size_t)P || srs->tables != srs->W) {  // one-shot bases: whole upload first
    fr_upload(ctx, d, h, n);
    return msm_device(ctx, srs, d, n);
  }
  if (!ctx->copy_stream) QG_HIP(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  // the hand-over events return to the pool only after the reduction's
  // synchronization (none is re-recorded while a queued wait refers to it)
  std::vector<hipEvent_t> held;
  {  // the uploads start after the work already queued on ctx->stream (stream
     // order in both directions: the scratch slot may still be read there)
    hipEvent_t ev = ctx->ev_get();
    held.push_back(ev);
    QG_HIP(hipEventRecord(ev, ctx->stream));
    QG_HIP(hipStreamWaitEvent(ctx->copy_stream, ev, 0));
  }
  std::vector<MsmRun> runs;
  const size_t per = div_up(n, (size_t)P);
  for (int k = 0; k < P; k++) {
    const size_t off = (size_t)k * per, len = std::min(per, n - std::min(n, off));
    if (len == 0) break;
    QG_HIP(hipMemcpyAsync(d + off, h + 4 * off, len * sizeof(Fr), hipMemcpyHostToDevice,
                          ctx->copy_stream));
    hipEvent_t ev = ctx->ev_get();
    held.push_back(ev);
    QG_HIP(hipEventRecord(ev, ctx->copy_stream));
    QG_HIP(hipStreamWaitEvent(ctx->stream, ev, 0));
    runs.push_back(msm_accumulate_phase(ctx, srs, d + off, len, k, off));
  }
  std::vector<G1Xyzz> part;
  msm_reduce_phase(ctx, srs, runs, part);  // ends with a synchronization
  for (hipEvent_t e : held) ctx->event_pool.push_back(e);
  G1Xyzz acc = G1Xyzz::infinity();
  for (const G1Xyzz& q : part) acc = xyzz_add(acc, q);
  return msm_finish_ranks(ctx, acc);
}

G1Affine msm_device(qg_ctx* ctx, const qg_srs* srs, const Fr* d_scalars, size_t n) {
  return msm_device_batch(ctx, srs, {d_scalars}, {n})[0];
}

// msm_unchecked over the base slice srs[off..] (qg_msm_g1_at / _dev_at): the
// entries point at rows off + i of each table (msm_accumulate_phase srs_off)
static G1Affine msm_device_at(qg_ctx* ctx, const qg_srs* srs, const Fr* d, size_t n, size_t off) {
  if (off == 0) return msm_device(ctx, srs, d, n);
  G1Xyzz acc = G1Xyzz::infinity();
  if (srs->tables != srs->W) {
    acc = msm_oneshot_local(ctx, srs, d, n, off);
  } else if (n > 0) {
    std::vector<MsmRun> runs{msm_accumulate_phase(ctx, srs, d, n, 0, off)};
    std::vector<G1Xyzz> part;
    msm_reduce_phase(ctx, srs, runs, part);  // ends with a synchronization
    acc = part[0];
  }
  return msm_finish_ranks(ctx, acc);
}

// dependent Fq multiply chains: 8 independent chains per thread, ITER steps
// Fq multiply throughput of the arithmetic the MSM runs (29-bit limbs)
__global__ void __launch_bounds__(256) k_fq_mul_bench(Fq* io, int iters) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Q29 a[4], b = to29(io[i & 1023]);
  for (int k = 0; k < 4; k++) a[k] = to29(io[(i + k + 1) & 1023]);
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = mul29(a[k], b);
  }
  uint32_t s = 0;
  for (int k = 0; k < 4; k++)
    for (int l = 0; l < 9; l++) s ^= a[k].l[l];
  if (s == 0x12345678u) io[i & 1023].v[0] = s;  // keep live
}

// FETCH_SIZE calibration (pmc_traffic.py): a known count of random table-row
// gathers in k_msm_accumulate's access pattern (five 16-B loads of one 128-B
// row per lane, msm_pt_load), and a 16-B-per-lane streaming read of the table
__global__ void __launch_bounds__(256) k_fetch_gather(const MsmPt* __restrict__ table, size_t rows,
                                                      size_t n, uint32_t* __restrict__ sink) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
  h ^= h >> 29;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 32;
  Q29 x, y;
  msm_pt_load(table, (uint32_t)(h % rows), (h >> 63) != 0, x, y);
  uint32_t s = 0;
#pragma unroll
  for (int l = 0; l < 9; l++) s ^= x.l[l] ^ y.l[l];
  sink[i] = s;
}

__global__ void __launch_bounds__(256) k_fetch_stream(const uint4* __restrict__ src, size_t n16,
                                                      uint32_t* __restrict__ sink) {
  const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t T = (size_t)gridDim.x * blockDim.x;
  uint32_t s = 0;
  for (size_t i = t; i < n16; i += T) {
    const uint4 v = src[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  sink[t] = s;
}

}  // namespace qg

extern "C" {

int qg_microbench_fetch(qg_ctx* ctx, size_t rows, size_t gathers, double* gather_ms,
                        double* stream_ms) {
  if (!ctx || !rows || !gathers || !gather_ms || !stream_ms || rows > 0xffffffffull)
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    MsmPt* table = ctx->scratch_as<MsmPt>("mb_fetch_table", rows);
    const unsigned sblocks = 256 * 8;
    uint32_t* sink = ctx->scratch_as<uint32_t>("mb_fetch_sink", std::max<size_t>(gathers, sblocks * 256));
    QG_HIP(hipMemsetAsync(table, 0x5a, rows * sizeof(MsmPt), ctx->stream));
    hipEvent_t a, b, c;
    QG_HIP(hipEventCreate(&a));
    QG_HIP(hipEventCreate(&b));
    QG_HIP(hipEventCreate(&c));
    QG_HIP(hipEventRecord(a, ctx->stream));
    hipLaunchKernelGGL(k_fetch_gather, dim3((unsigned)div_up(gathers, (size_t)256)), dim3(256), 0,
                       ctx->stream, table, rows, gathers, sink);
    QG_LAUNCH_CHECK();
    QG_HIP(hipEventRecord(b, ctx->stream));
    hipLaunchKernelGGL(k_fetch_stream, dim3(sblocks), dim3(256), 0, ctx->stream,
                       reinterpret_cast<const uint4*>(table), rows * sizeof(MsmPt) / 16, sink);
    QG_LAUNCH_CHECK();
    QG_HIP(hipEventRecord(c, ctx->stream));
    QG_HIP(hipEventSynchronize(c));
    float m1 = 0, m2 = 0;
    QG_HIP(hipEventElapsedTime(&m1, a, b));
    QG_HIP(hipEventElapsedTime(&m2, b, c));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipEventDestroy(c);
    *gather_ms = m1;
    *stream_ms = m2;
  });
}

int qg_microbench_fq_mul(qg_ctx* ctx, double* mul_per_s) {
  if (!ctx || !mul_per_s) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    Fq* io = ctx->scratch_as<Fq>("mb_io", 1024);
    std::vector<Fq> h(1024);
    for (int i = 0; i < 1024; i++) h[i] = from_u64<FqP>(1000003ull * (i + 7));
    QG_HIP(hipMemcpyAsync(io, h.data(), sizeof(Fq) * 1024, hipMemcpyHostToDevice, ctx->stream));
    const int iters = 2048;
    const unsigned blocks = 256 * 16;  // 16 blocks of 4 waves per CU
    hipEvent_t a, b;
    QG_HIP(hipEventCreate(&a));
    QG_HIP(hipEventCreate(&b));
    hipLaunchKernelGGL(k_fq_mul_bench, dim3(blocks), dim3(256), 0, ctx->stream, io, 64);  // warm
    QG_HIP(hipEventRecord(a, ctx->stream));
    hipLaunchKernelGGL(k_fq_mul_bench, dim3(blocks), dim3(256), 0, ctx->stream, io, iters);
    QG_HIP(hipEventRecord(b, ctx->stream));
    QG_HIP(hipEventSynchronize(b));
    float ms = 0;
    QG_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *mul_per_s = (double)blocks * 256.0 * 4.0 * iters / (ms * 1e-3);
  });
}

static int srs_upload_impl(qg_ctx* ctx, const uint64_t* affine_xy, const uint8_t* infinity, size_t n,
                           bool oneshot, qg_srs** out) {
  if (!ctx || !out || (!affine_xy && n)) return QG_ERR_INVALID;
  *out = nullptr;
  qg_srs* srs = nullptr;
  int rc = qg_guard(ctx, [&] {
    QG_CHECK(n > 0, QG_ERR_INVALID, "empty SRS");
    QG_HIP(hipSetDevice(ctx->device));
    srs = srs_alloc(ctx, n, oneshot);
    uint64_t* d_xy = ctx->scratch_as<uint64_t>("srs_up_xy", n * 8);
    uint8_t* d_inf = nullptr;
    QG_HIP(hipMemcpyAsync(d_xy, affine_xy, n * 64, hipMemcpyHostToDevice, ctx->stream));
    if (infinity) {
      d_inf = ctx->scratch_as<uint8_t>("srs_up_inf", n);
      QG_HIP(hipMemcpyAsync(d_inf, infinity, n, hipMemcpyHostToDevice, ctx->stream));
    }
    G1Affine* d_base = ctx->scratch_as<G1Affine>("srs_base", n);
    hipLaunchKernelGGL(k_import_bases, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_xy,
                       d_inf, n, d_base);
    QG_LAUNCH_CHECK();
    srs_build_tables(ctx, srs, d_base);
    ctx->sync();
  });
  if (rc != QG_OK) {
    if (srs) {
      (void)hipFree(srs->d_table);
      delete srs;
    }
    return rc;
  }
  *out = srs;
  return QG_OK;
}

int qg_srs_upload(qg_ctx* ctx, const uint64_t* affine_xy, const uint8_t* infinity, size_t n,
                  qg_srs** out) {
  return srs_upload_impl(ctx, affine_xy, infinity, n, false, out);
}

int qg_bases_upload(qg_ctx* ctx, const uint64_t* affine_xy, const uint8_t* infinity, size_t n,
                    qg_srs** out) {
  return srs_upload_impl(ctx, affine_xy, infinity, n, true, out);
}

int qg_srs_generate(qg_ctx* ctx, const uint64_t tau[4], const uint64_t* g_xy, size_t n,
                    qg_srs** out) {
  return qg_srs_generate_range(ctx, tau, g_xy, 0, n, out);
}

int qg_srs_generate_range(qg_ctx* ctx, const uint64_t tau[4], const uint64_t* g_xy,
                          uint64_t offset, size_t n, qg_srs** out) {
  if (!ctx || !out || !tau) return QG_ERR_INVALID;
  *out = nullptr;
  qg_srs* srs = nullptr;
  int rc = qg_guard(ctx, [&] {
    QG_CHECK(n > 0, QG_ERR_INVALID, "empty SRS");
    QG_HIP(hipSetDevice(ctx->device));
    srs = srs_alloc(ctx, n);
    G1Affine g;
    if (g_xy) {
      g = g1_import(g_xy, 0);
    } else {
      g.x = from_u64<FqP>(1);
      g.y = from_u64<FqP>(2);
    }
    Fr t = fr_import(tau);
    Fr* d_pow = ctx->scratch_as<Fr>("srs_pow", n);
    G1Xyzz* d_fbb = ctx->scratch_as<G1Xyzz>("srs_fbb", 32);
    G1Affine* d_fb = ctx->scratch_as<G1Affine>("srs_fb", 32 * 256);
    G1Affine* d_base = ctx->scratch_as<G1Affine>("srs_base", n);
    {
      QgTimed tm(ctx, "srs_generate");
      const int K = 64;
      hipLaunchKernelGGL(k_powers, dim3(div_up(div_up(n, K), 256)), dim3(256), 0, ctx->stream, t,
                         offset, n, K, d_pow);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_fb_powers, dim3(1), dim3(64), 0, ctx->stream, g, d_fbb);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_fb_table, dim3(32), dim3(256), 0, ctx->stream, d_fbb, d_fb);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_fb_mul, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_fb, d_pow,
                         n, d_base);
      QG_LAUNCH_CHECK();
    }
    srs_build_tables(ctx, srs, d_base);
    ctx->sync();
  });
  if (rc != QG_OK) {
    if (srs) {
      (void)hipFree(srs->d_table);
      delete srs;
    }
    return rc;
  }
  *out = srs;
  return QG_OK;
}

int qg_srs_destroy(qg_srs* srs) {
  if (!srs) return QG_OK;
  (void)hipFree(srs->d_table);
  delete srs;
  return QG_OK;
}

size_t qg_srs_len(const qg_srs* srs) { return srs ? srs->n : 0; }

int qg_srs_window_info(const qg_srs* srs, int* c, int* windows) {
  if (!srs) return QG_ERR_INVALID;
  if (c) *c = srs->c;
  if (windows) *windows = srs->W;
  return QG_OK;
}

int qg_srs_download(const qg_srs* srs, size_t offset, size_t n, uint64_t* affine_xy,
                    uint8_t* infinity) {
  if (!srs || (!affine_xy && n) || offset + n > srs->n) return QG_ERR_INVALID;
  qg_ctx* ctx = srs->ctx;
  return qg_guard(ctx, [&] {
    if (n == 0) return;
    QG_HIP(hipSetDevice(ctx->device));
    std::vector<G1Affine> h(n);
    G1Affine* d = ctx->scratch_as<G1Affine>("srs_download", n);
    hipLaunchKernelGGL(k_srs_unpack, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream,
                       srs->d_table + offset, n, d);
    QG_LAUNCH_CHECK();
    QG_HIP(hipMemcpyAsync(h.data(), d, n * sizeof(G1Affine), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    for (size_t i = 0; i < n; i++) g1_export(h[i], affine_xy + 8 * i, infinity ? infinity + i : nullptr);
  });
}

int qg_msm_g1_dev(qg_ctx* ctx, const qg_srs* srs, const qg_buf* scalars, size_t n,
                  uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || !scalars || !out_xy || n > scalars->n) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    G1Affine r = msm_device(ctx, srs, scalars->d, n);
    g1_export(r, out_xy, out_inf);
  });
}

int qg_msm_g1_dev_at(qg_ctx* ctx, const qg_srs* srs, size_t offset, const qg_buf* scalars,
                     size_t n, uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || !scalars || !out_xy || n > scalars->n || offset > srs->n)
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    const size_t m = std::min(n, srs->n - offset);  // msm_unchecked truncation
    g1_export(msm_device_at(ctx, srs, scalars->d, m, offset), out_xy, out_inf);
  });
}

int qg_msm_g1_at(qg_ctx* ctx, const qg_srs* srs, size_t offset, const uint64_t* scalars,
                 size_t n, uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || (!scalars && n) || !out_xy || offset > srs->n) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    const size_t m = std::min(n, srs->n - offset);
    Fr* d = ctx->scratch_as<Fr>("msm_scalars", m ? m : 1);
    fr_upload(ctx, d, scalars, m);
    g1_export(msm_device_at(ctx, srs, d, m, offset), out_xy, out_inf);
  });
}

int qg_msm_g1_dev_batch(qg_ctx* ctx, const qg_srs* srs, const qg_buf* const* scalars,
                        const size_t* ns, size_t k, uint64_t* out_xy, uint8_t* out_inf) {
  if (!ctx || !srs || (k && (!scalars || !ns || !out_xy || !out_inf))) return QG_ERR_INVALID;
  for (size_t i = 0; i < k; i++)
    if (!scalars[i] || ns[i] > scalars[i]->n) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(k <= (size_t)MSM_MAX_BATCH, QG_ERR_UNSUPPORTED, "MSM batch too large");
    QG_HIP(hipSetDevice(ctx->device));
    std::vector<const Fr*> sc(k);
    std::vector<size_t> n(k);
    for (size_t i = 0; i < k; i++) {
      sc[i] = scalars[i]->d;
      n[i] = ns[i];
    }
    const std::vector<G1Affine> r = msm_device_batch(ctx, srs, sc, n);
    for (size_t i = 0; i < k; i++) g1_export(r[i], out_xy + 8 * i, out_inf + i);
  });
}

int qg_msm_g1(qg_ctx* ctx, const qg_srs* srs, const uint64_t* scalars, size_t n,
              uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || (!scalars && n) || !out_xy) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    // msm_unchecked truncates to min(len(bases), len(scalars))
    size_t m = n < srs->n ? n : srs->n;
    G1Affine r = msm_host(ctx, srs, scalars, m);
    g1_export(r, out_xy, out_inf);
  });
}

int qg_kzg_commit(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n,
                  uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || (!poly && n) || !out_xy) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(n <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
    QG_HIP(hipSetDevice(ctx->device));
    G1Affine r = msm_host(ctx, srs, poly, n);
    g1_export(r, out_xy, out_inf);
  });
}

}  // extern "C"
