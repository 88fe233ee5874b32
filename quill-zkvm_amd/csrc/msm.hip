// Pippenger MSM over BN254 G1 for gfx950 — replaces
// `E::G1::msm_unchecked(&g1_points_affine, polynomial)` at pcs/src/kzg.rs:72
// (ark-ec 0.5.0 VariableBaseMSM) and the SRS handling of KZG::commit
// (kzg.rs:61-73) / KZG::trusted_setup (kzg.rs:35-59).
//
// Design (MI355X-first; see DESIGN.md "MSM"):
//  * The SRS lives in HBM as affine points (64 B each, (0,0) = infinity) together
//    with W-1 window-shifted copies table[w][i] = 2^(c*w) * P_i.  288 GB of HBM
//    makes this cheap (2^24 bases, c = 21: 13 tables, 14 GB) and it removes the
//    serial window-combination doublings: every signed c-bit digit of every
//    scalar lands in ONE shared set of 2^(c-1) buckets.
//  * Bucketing is a counting sort: count (atomics) -> scan -> scatter (atomics).
//    Digits are recomputed from the scalars in the scatter pass (32 B/scalar)
//    instead of materializing n*W keys.
//  * Accumulation is load-balanced: every bucket is split into chunks of
//    E entries, one thread per chunk, so skewed digit distributions (small
//    witness values, the short top window) do not serialize on one lane.
//    Mixed XYZZ + affine additions (8M + 2S), no inversions.
//  * Bucket reduction sum_j (j+1) B_j runs as independent running sums over
//    segments of L buckets; segment s contributes acc_s + lo_s * run_s; blocks
//    tree-reduce in LDS; one final block sums block results.
#include "common.h"

using namespace qg;

namespace qg {

static constexpr int MSM_E = 32;        // entries per accumulation thread
static constexpr int MSM_SEG = 16;      // buckets per reduction segment
static constexpr int MSM_BLOCK = 256;

// window size for an SRS of n bases (tuned later)
static int msm_window_bits(size_t n) {
  int lg = 0;
  while (((size_t)1 << lg) < n) lg++;
  int c = lg - 3;
  if (c < 4) c = 4;
  if (c > 21) c = 21;
  return c;
}

QG_DEV uint32_t scalar_bits(const uint32_t s[8], int lo, int c) {
  if (lo >= 256) return 0;
  int li = lo >> 5, sh = lo & 31;
  uint64_t w = s[li];
  if (li + 1 < 8) w |= (uint64_t)s[li + 1] << 32;
  return (uint32_t)(w >> sh) & ((1u << c) - 1u);
}

// signed c-bit digit decomposition, emit(w, bucket, neg) for nonzero digits
template <class Emit>
QG_DEV void for_each_digit(const Fr& mont_scalar, int c, int W, Emit&& emit) {
  Fr s = from_mont(mont_scalar);
  const uint32_t half = 1u << (c - 1);
  const uint32_t full = 1u << c;
  uint32_t carry = 0;
  for (int w = 0; w < W; w++) {
    uint32_t d = scalar_bits(s.v, w * c, c) + carry;
    if (d > half) {
      carry = 1;
      uint32_t mag = full - d;  // digit = d - 2^c < 0
      if (mag) emit(w, mag - 1, true);
    } else {
      carry = 0;
      if (d) emit(w, d - 1, false);
    }
  }
}

__global__ void k_msm_count(const Fr* __restrict__ scalars, size_t n, int c, int W,
                            uint32_t* __restrict__ counts) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for_each_digit(scalars[i], c, W, [&](int, uint32_t b, bool) { atomicAdd(&counts[b], 1u); });
}

__global__ void k_msm_scatter(const Fr* __restrict__ scalars, size_t n, size_t N, int c, int W,
                              uint32_t* __restrict__ cursor, uint32_t* __restrict__ entries) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  for_each_digit(scalars[i], c, W, [&](int w, uint32_t b, bool neg) {
    uint32_t pos = atomicAdd(&cursor[b], 1u);
    entries[pos] = (uint32_t)((size_t)w * N + i) | (neg ? 0x80000000u : 0u);
  });
}

// ---- exclusive scan of (count, ceil(count/E)) over nb buckets -------------
static constexpr int SCAN_PER_THREAD = 8;
static constexpr int SCAN_BLOCK = 256;
static constexpr int SCAN_TILE = SCAN_PER_THREAD * SCAN_BLOCK;

__device__ __forceinline__ uint2 scan_val(const uint32_t* counts, size_t i, size_t nb) {
  uint32_t c = i < nb ? counts[i] : 0u;
  return make_uint2(c, (c + MSM_E - 1) / MSM_E);
}

// per-tile exclusive scan; writes tile totals
__global__ void k_scan_tiles(const uint32_t* __restrict__ counts, size_t nb,
                             uint32_t* __restrict__ bstart, uint32_t* __restrict__ tstart,
                             uint2* __restrict__ tile_tot) {
  __shared__ uint2 sh[SCAN_BLOCK];
  size_t base = (size_t)blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_PER_THREAD;
  uint2 v[SCAN_PER_THREAD];
  uint2 tot = make_uint2(0, 0);
  for (int k = 0; k < SCAN_PER_THREAD; k++) {
    v[k] = scan_val(counts, base + k, nb);
    tot.x += v[k].x;
    tot.y += v[k].y;
  }
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
    if (i < nb) {
      bstart[i] = run.x;
      tstart[i] = run.y;
    }
    run.x += v[k].x;
    run.y += v[k].y;
  }
  if (threadIdx.x == SCAN_BLOCK - 1) tile_tot[blockIdx.x] = sh[SCAN_BLOCK - 1];
}

// single block: exclusive scan of tile totals (ntiles <= 1024 * 8)
__global__ void k_scan_top(uint2* __restrict__ tile_tot, int ntiles, uint32_t* __restrict__ bstart,
                           uint32_t* __restrict__ tstart, size_t nb) {
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
  if (threadIdx.x == 1023) {
    bstart[nb] = sh[1023].x;
    tstart[nb] = sh[1023].y;
  }
}

__global__ void k_scan_add(const uint2* __restrict__ tile_off, size_t nb, uint32_t* __restrict__ bstart,
                           uint32_t* __restrict__ tstart, uint32_t* __restrict__ cursor) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nb) return;
  uint2 off = tile_off[i / SCAN_TILE];
  uint32_t b = bstart[i] + off.x;
  bstart[i] = b;
  cursor[i] = b;
  tstart[i] += off.y;
}

// ---- accumulation ---------------------------------------------------------
__global__ void __launch_bounds__(MSM_BLOCK)
    k_msm_accumulate(const G1Affine* __restrict__ table, const uint32_t* __restrict__ entries,
                     const uint32_t* __restrict__ bstart, const uint32_t* __restrict__ tstart,
                     uint32_t nb, G1Xyzz* __restrict__ partial) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t total = tstart[nb];
  if (t >= total) return;
  // bucket b: largest with tstart[b] <= t
  uint32_t lo = 0, hi = nb;
  while (hi - lo > 1) {
    uint32_t mid = (lo + hi) >> 1;
    if (tstart[mid] <= t) lo = mid;
    else hi = mid;
  }
  const uint32_t b = lo;
  const uint32_t e0 = bstart[b] + (t - tstart[b]) * MSM_E;
  uint32_t e1 = e0 + MSM_E;
  const uint32_t bend = bstart[b + 1];
  if (e1 > bend) e1 = bend;
  G1Xyzz acc = G1Xyzz::infinity();
  for (uint32_t e = e0; e < e1; e++) {
    const uint32_t ent = entries[e];
    G1Affine p = table[ent & 0x7fffffffu];
    if (ent >> 31) p.y = fneg(p.y);
    acc = xyzz_add_affine(acc, p);
  }
  partial[t] = acc;
}

// ---- reduction ------------------------------------------------------------
__device__ void block_reduce_xyzz(G1Xyzz v, G1Xyzz* sh, G1Xyzz* out) {
  sh[threadIdx.x] = v;
  __syncthreads();
  for (unsigned s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) sh[threadIdx.x] = xyzz_add(sh[threadIdx.x], sh[threadIdx.x + s]);
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = sh[0];
}

__global__ void __launch_bounds__(MSM_BLOCK)
    k_msm_reduce(const G1Xyzz* __restrict__ partial, const uint32_t* __restrict__ tstart,
                 uint32_t nb, G1Xyzz* __restrict__ block_out) {
  __shared__ G1Xyzz sh[MSM_BLOCK];
  const uint32_t seg = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lo = seg * MSM_SEG;
  G1Xyzz v = G1Xyzz::infinity();
  if (lo < nb) {
    uint32_t hi = lo + MSM_SEG < nb ? lo + MSM_SEG : nb;
    G1Xyzz run = G1Xyzz::infinity(), acc = G1Xyzz::infinity();
    for (uint32_t j = hi; j-- > lo;) {
      const uint32_t t0 = tstart[j], t1 = tstart[j + 1];
      for (uint32_t t = t0; t < t1; t++) run = xyzz_add(run, partial[t]);
      acc = xyzz_add(acc, run);
    }
    // bucket j has weight j+1 = (j - lo + 1) + lo
    v = xyzz_add(acc, xyzz_mul_small(run, lo));
  }
  block_reduce_xyzz(v, sh, &block_out[blockIdx.x]);
}

__global__ void __launch_bounds__(MSM_BLOCK)
    k_msm_final(const G1Xyzz* __restrict__ in, uint32_t m, G1Xyzz* __restrict__ out) {
  __shared__ G1Xyzz sh[MSM_BLOCK];
  G1Xyzz v = G1Xyzz::infinity();
  for (uint32_t i = threadIdx.x; i < m; i += blockDim.x) v = xyzz_add(v, in[i]);
  block_reduce_xyzz(v, sh, out);
}

// ---- SRS construction -----------------------------------------------------
// table[w*N + i] = 2^c * table[(w-1)*N + i]
__global__ void k_srs_shift(G1Affine* table, size_t N, int w, int c) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  G1Affine a = table[(size_t)(w - 1) * N + i];
  G1Xyzz p = G1Xyzz::from_affine(a);
  for (int k = 0; k < c; k++) p = xyzz_dbl(p);
  table[(size_t)w * N + i] = xyzz_to_affine(p);
}

// tau^(offset+i) for i < n, K consecutive powers per thread
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

static void srs_build_shifts(qg_ctx* ctx, qg_srs* srs) {
  QgTimed tm(ctx, "srs_shift");
  for (int w = 1; w < srs->W; w++) {
    hipLaunchKernelGGL(k_srs_shift, dim3(div_up(srs->n, 256)), dim3(256), 0, ctx->stream,
                       srs->d_table, srs->n, w, srs->c);
    QG_LAUNCH_CHECK();
  }
}

static qg_srs* srs_alloc(qg_ctx* ctx, size_t n) {
  qg_srs* srs = new qg_srs();
  srs->ctx = ctx;
  srs->n = n;
  srs->c = msm_window_bits(n);
  srs->W = (255 + srs->c - 1) / srs->c;
  hipError_t e = hipMalloc(&srs->d_table, (size_t)srs->W * n * sizeof(G1Affine));
  if (e != hipSuccess) {
    delete srs;
    throw Error(QG_ERR_OOM, "qg_srs: hipMalloc of the window tables failed");
  }
  return srs;
}

G1Affine msm_device(qg_ctx* ctx, const qg_srs* srs, const Fr* d_scalars, size_t n) {
  QG_CHECK(n <= srs->n, QG_ERR_INVALID, "MSM length exceeds the SRS");
  G1Xyzz local = G1Xyzz::infinity();
  if (n > 0) {
    const int c = srs->c, W = srs->W;
    const uint32_t nb = 1u << (c - 1);
    const size_t max_entries = n * (size_t)W;
    QG_CHECK((size_t)W * srs->n < 0x80000000ull, QG_ERR_UNSUPPORTED, "SRS table index overflow");
    QG_CHECK(max_entries < 0xffffffffull, QG_ERR_UNSUPPORTED, "too many MSM entries");
    uint32_t* counts = ctx->scratch_as<uint32_t>("msm_counts", nb);
    uint32_t* bstart = ctx->scratch_as<uint32_t>("msm_bstart", nb + 1);
    uint32_t* tstart = ctx->scratch_as<uint32_t>("msm_tstart", nb + 1);
    uint32_t* cursor = ctx->scratch_as<uint32_t>("msm_cursor", nb);
    uint32_t* entries = ctx->scratch_as<uint32_t>("msm_entries", max_entries + 1);
    const int ntiles = (int)div_up(nb, SCAN_TILE);
    uint2* tile_tot = ctx->scratch_as<uint2>("msm_tiles", ntiles);
    const size_t max_threads = max_entries / MSM_E + nb + 1;
    G1Xyzz* partial = ctx->scratch_as<G1Xyzz>("msm_partial", max_threads);
    const uint32_t nseg = div_up(nb, MSM_SEG);
    const uint32_t nred = div_up(nseg, MSM_BLOCK);
    G1Xyzz* red = ctx->scratch_as<G1Xyzz>("msm_red", nred + 1);
    QG_CHECK(ntiles <= 1024 * 64, QG_ERR_UNSUPPORTED, "bucket count too large");

    {
      QgTimed tm(ctx, "msm_bucketing");
      QG_HIP(hipMemsetAsync(counts, 0, nb * sizeof(uint32_t), ctx->stream));
      hipLaunchKernelGGL(k_msm_count, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_scalars,
                         n, c, W, counts);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan_tiles, dim3(ntiles), dim3(SCAN_BLOCK), 0, ctx->stream, counts,
                         (size_t)nb, bstart, tstart, tile_tot);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, ctx->stream, tile_tot, ntiles,
                         bstart, tstart, (size_t)nb);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_scan_add, dim3(div_up(nb, 256)), dim3(256), 0, ctx->stream, tile_tot,
                         (size_t)nb, bstart, tstart, cursor);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_msm_scatter, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream,
                         d_scalars, n, srs->n, c, W, cursor, entries);
      QG_LAUNCH_CHECK();
    }
    {
      QgTimed tm(ctx, "msm_accumulate");
      hipLaunchKernelGGL(k_msm_accumulate, dim3(div_up(max_threads, MSM_BLOCK)), dim3(MSM_BLOCK),
                         0, ctx->stream, srs->d_table, entries, bstart, tstart, nb, partial);
      QG_LAUNCH_CHECK();
    }
    {
      QgTimed tm(ctx, "msm_reduce");
      hipLaunchKernelGGL(k_msm_reduce, dim3(nred), dim3(MSM_BLOCK), 0, ctx->stream, partial,
                         tstart, nb, red);
      QG_LAUNCH_CHECK();
      hipLaunchKernelGGL(k_msm_final, dim3(1), dim3(MSM_BLOCK), 0, ctx->stream, red, nred,
                         red + nred);
      QG_LAUNCH_CHECK();
    }
    QG_HIP(hipMemcpyAsync(&local, red + nred, sizeof(G1Xyzz), hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
  }
  if (ctx->world > 1) {
    // sum of the per-rank partial MSMs (allgather + host EC adds; RCCL cannot add points)
    G1Xyzz* d_send = ctx->scratch_as<G1Xyzz>("msm_comm_send", 1);
    G1Xyzz* d_recv = ctx->scratch_as<G1Xyzz>("msm_comm_recv", ctx->world);
    QG_HIP(hipMemcpyAsync(d_send, &local, sizeof(G1Xyzz), hipMemcpyHostToDevice, ctx->stream));
    comm_allgather_bytes(ctx, d_send, d_recv, sizeof(G1Xyzz));
    std::vector<G1Xyzz> all(ctx->world);
    QG_HIP(hipMemcpyAsync(all.data(), d_recv, sizeof(G1Xyzz) * ctx->world, hipMemcpyDeviceToHost,
                          ctx->stream));
    ctx->sync();
    local = G1Xyzz::infinity();
    for (int r = 0; r < ctx->world; r++) local = xyzz_add(local, all[r]);
  }
  return xyzz_to_affine(local);
}

// dependent Fq multiply chains: 8 independent chains per thread, ITER steps
__global__ void __launch_bounds__(256) k_fq_mul_bench(Fq* io, int iters) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  Fq a[4], b = io[i & 1023];
  for (int k = 0; k < 4; k++) a[k] = io[(i + k + 1) & 1023];
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int k = 0; k < 4; k++) a[k] = a[k] * b;
  }
  Fq s = a[0] + a[1] + a[2] + a[3];
  if (s.v[0] == 0x12345678u) io[i & 1023] = s;  // keep live
}

}  // namespace qg

extern "C" {

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

int qg_srs_upload(qg_ctx* ctx, const uint64_t* affine_xy, const uint8_t* infinity, size_t n,
                  qg_srs** out) {
  if (!ctx || !out || (!affine_xy && n)) return QG_ERR_INVALID;
  *out = nullptr;
  qg_srs* srs = nullptr;
  int rc = qg_guard(ctx, [&] {
    QG_CHECK(n > 0, QG_ERR_INVALID, "empty SRS");
    QG_HIP(hipSetDevice(ctx->device));
    srs = srs_alloc(ctx, n);
    uint64_t* d_xy = ctx->scratch_as<uint64_t>("srs_up_xy", n * 8);
    uint8_t* d_inf = nullptr;
    QG_HIP(hipMemcpyAsync(d_xy, affine_xy, n * 64, hipMemcpyHostToDevice, ctx->stream));
    if (infinity) {
      d_inf = ctx->scratch_as<uint8_t>("srs_up_inf", n);
      QG_HIP(hipMemcpyAsync(d_inf, infinity, n, hipMemcpyHostToDevice, ctx->stream));
    }
    hipLaunchKernelGGL(k_import_bases, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream, d_xy,
                       d_inf, n, srs->d_table);
    QG_LAUNCH_CHECK();
    srs_build_shifts(ctx, srs);
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
                         n, srs->d_table);
      QG_LAUNCH_CHECK();
    }
    srs_build_shifts(ctx, srs);
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

int qg_srs_download(const qg_srs* srs, size_t offset, size_t n, uint64_t* affine_xy,
                    uint8_t* infinity) {
  if (!srs || (!affine_xy && n) || offset + n > srs->n) return QG_ERR_INVALID;
  qg_ctx* ctx = srs->ctx;
  return qg_guard(ctx, [&] {
    std::vector<G1Affine> h(n);
    QG_HIP(hipMemcpyAsync(h.data(), srs->d_table + offset, n * sizeof(G1Affine),
                          hipMemcpyDeviceToHost, ctx->stream));
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

int qg_msm_g1(qg_ctx* ctx, const qg_srs* srs, const uint64_t* scalars, size_t n,
              uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || (!scalars && n) || !out_xy) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    // msm_unchecked truncates to min(len(bases), len(scalars))
    size_t m = n < srs->n ? n : srs->n;
    Fr* d = ctx->scratch_as<Fr>("msm_scalars", m ? m : 1);
    fr_upload(ctx, d, scalars, m);
    G1Affine r = msm_device(ctx, srs, d, m);
    g1_export(r, out_xy, out_inf);
  });
}

int qg_kzg_commit(qg_ctx* ctx, const qg_srs* srs, const uint64_t* poly, size_t n,
                  uint64_t out_xy[8], uint8_t* out_inf) {
  if (!ctx || !srs || (!poly && n) || !out_xy) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_CHECK(n <= srs->n, QG_ERR_INVALID, "Polynomial degree exceeds max degree");
    QG_HIP(hipSetDevice(ctx->device));
    Fr* d = ctx->scratch_as<Fr>("msm_scalars", n ? n : 1);
    fr_upload(ctx, d, poly, n);
    G1Affine r = msm_device(ctx, srs, d, n);
    g1_export(r, out_xy, out_inf);
  });
}

}  // extern "C"
