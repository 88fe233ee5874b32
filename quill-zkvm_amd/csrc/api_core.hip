// C-ABI core: context, transcript, serialization, device Fr vectors.
#include <atomic>
#include <string.h>

#include "blake3.h"
#include <algorithm>

#include "common.h"

using namespace qg;

namespace qg {

Fr fr_import(const uint64_t v[4]) {
  Fr r;
  for (int i = 0; i < 4; i++) {
    r.v[2 * i] = (uint32_t)v[i];
    r.v[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
  return r;
}

void fr_export(const Fr& a, uint64_t v[4]) {
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
}

static Fq fq_import(const uint64_t v[4]) {
  Fq r;
  for (int i = 0; i < 4; i++) {
    r.v[2 * i] = (uint32_t)v[i];
    r.v[2 * i + 1] = (uint32_t)(v[i] >> 32);
  }
  return r;
}

static void fq_export(const Fq& a, uint64_t v[4]) {
  for (int i = 0; i < 4; i++) v[i] = (uint64_t)a.v[2 * i] | ((uint64_t)a.v[2 * i + 1] << 32);
}

void g1_export(const G1Affine& a, uint64_t xy[8], uint8_t* inf) {
  if (a.is_inf()) {
    memset(xy, 0, 64);
    if (inf) *inf = 1;
    return;
  }
  fq_export(a.x, xy);
  fq_export(a.y, xy + 4);
  if (inf) *inf = 0;
}

G1Affine g1_import(const uint64_t xy[8], uint8_t inf) {
  if (inf) return G1Affine::infinity();
  return {fq_import(xy), fq_import(xy + 4)};
}

// ark-serialize SW uncompressed: x || y (canonical LE), flags in y's top byte:
// bit 7 = y > -y ("negative"), bit 6 = infinity (x = y = 0).
void g1_serialize(const G1Affine& a, uint8_t out[64]) {
  memset(out, 0, 64);
  if (a.is_inf()) {
    out[63] |= 0x40;
    return;
  }
  Fq x = from_mont(a.x), y = from_mont(a.y);
  Fq ny = from_mont(fneg(a.y));
  for (int i = 0; i < 8; i++)
    for (int b = 0; b < 4; b++) {
      out[4 * i + b] = (uint8_t)(x.v[i] >> (8 * b));
      out[32 + 4 * i + b] = (uint8_t)(y.v[i] >> (8 * b));
    }
  if (limbs_gt(y.v, ny.v)) out[63] |= 0x80;
}

void fr_upload(qg_ctx* ctx, Fr* d, const uint64_t* h, size_t n) {
  if (n == 0) return;
  QG_HIP(hipMemcpyAsync(d, h, n * 32, hipMemcpyHostToDevice, ctx->stream));
}

void fr_download(qg_ctx* ctx, uint64_t* h, const Fr* d, size_t n) {
  if (n == 0) return;
  QG_HIP(hipMemcpyAsync(h, d, n * 32, hipMemcpyDeviceToHost, ctx->stream));
}

// splitmix64 -> xoshiro256** per 64-element block; Fr sampled as 4 LE u64,
// top limb masked to 62 bits, rejected if >= r (uniform), then to Montgomery.
__global__ void k_fill_random(Fr* out, size_t n, uint64_t seed) {
  size_t blk = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t base = blk * 64;
  if (base >= n) return;
  uint64_t s = seed ^ (0x9E3779B97F4A7C15ull * (blk + 1));
  uint64_t st[4];
  for (int i = 0; i < 4; i++) {
    s += 0x9E3779B97F4A7C15ull;
    uint64_t z = s;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    st[i] = z ^ (z >> 31);
  }
  auto next = [&]() {
    uint64_t r = ((st[1] * 5) << 7 | (st[1] * 5) >> 57) * 9;
    uint64_t t = st[1] << 17;
    st[2] ^= st[0];
    st[3] ^= st[1];
    st[1] ^= st[2];
    st[0] ^= st[3];
    st[2] ^= t;
    st[3] = (st[3] << 45) | (st[3] >> 19);
    return r;
  };
  size_t end = base + 64 < n ? base + 64 : n;
  for (size_t i = base; i < end; i++) {
    Fr v;
    for (;;) {
      for (int l = 0; l < 4; l++) {
        uint64_t x = next();
        if (l == 3) x &= (1ull << 62) - 1;
        v.v[2 * l] = (uint32_t)x;
        v.v[2 * l + 1] = (uint32_t)(x >> 32);
      }
      bool lt = limbs_gt(FrP::P, v.v);
      if (lt) break;
    }
    out[i] = to_mont(v);
  }
}

// F::from(u64) for small integers (index mappings, transition_circuit.rs:120-151)
__global__ void k_from_u64(Fr* out, const uint64_t* v, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Fr x;
  for (int l = 0; l < 8; l++) x.v[l] = 0;
  x.v[0] = (uint32_t)v[i];
  x.v[1] = (uint32_t)(v[i] >> 32);
  out[i] = to_mont(x);
}

// canonical 4 x u64 LE -> Montgomery in place; flags values >= r
__global__ void k_canon_to_mont(Fr* io, size_t n, uint32_t* err) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr x = io[i];
  if (!limbs_gt(FrP::P, x.v)) {
    atomicOr(err, 1u);
    return;
  }
  io[i] = to_mont(x);
}

// first index i < n with a[i] != b[i] (atomicMin; n if none)
__global__ void k_first_mismatch(const Fr* a, const Fr* b, size_t n, unsigned long long* first) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fr x = a[i], y = b[i];
  bool eq = true;
  for (int l = 0; l < 8; l++) eq &= x.v[l] == y.v[l];
  if (!eq) atomicMin(first, (unsigned long long)i);
}

// profiling marker (qg_trace_marker): no work, only a dispatch whose grid
// size carries the caller's tag into the kernel trace
__global__ void k_trace_marker() {}

}  // namespace qg

extern "C" {

const char* qg_version(void) { return "quill_gpu 0.1 gfx950"; }

int qg_ctx_create(int device, qg_ctx** out) {
  if (!out) return QG_ERR_INVALID;
  *out = nullptr;
  qg_ctx* ctx = new qg_ctx();
  ctx->arena.backend.drain = &qg_ctx::drain_streams;
  ctx->arena.backend.owner = ctx;
  int rc = qg_guard(ctx, [&] {
    int ndev = 0;
    QG_HIP(hipGetDeviceCount(&ndev));
    QG_CHECK(device >= 0 && device < ndev, QG_ERR_INVALID, "no such HIP device");
    ctx->device = device;
    QG_HIP(hipSetDevice(device));
    QG_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  });
  if (rc != QG_OK) {
    delete ctx;
    return rc;
  }
  *out = ctx;
  return QG_OK;
}

int qg_ctx_destroy(qg_ctx* ctx) {
  if (!ctx) return QG_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->copy_stream) (void)hipStreamSynchronize(ctx->copy_stream);
  if (ctx->side_stream) (void)hipStreamSynchronize(ctx->side_stream);
  if (ctx->side_stream2) (void)hipStreamSynchronize(ctx->side_stream2);
  comm_release(ctx);
  try {
    ctx->arena.release_all();
  } catch (...) {  // destroy frees what it can; errors were reported by the calls before
  }
  for (auto& kv : ctx->pinned) (void)hipHostFree(kv.second.first);
  for (auto& kv : ctx->pending) {
    (void)hipEventDestroy(kv.second.a);
    (void)hipEventDestroy(kv.second.b);
  }
  for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
  if (ctx->tref) (void)hipEventDestroy(ctx->tref);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->copy_stream) (void)hipStreamDestroy(ctx->copy_stream);
  if (ctx->side_stream) (void)hipStreamDestroy(ctx->side_stream);
  if (ctx->side_stream2) (void)hipStreamDestroy(ctx->side_stream2);
  delete ctx;
  return QG_OK;
}

const char* qg_last_error(const qg_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

int qg_ctx_enable_timing(qg_ctx* ctx, int enable) {
  if (!ctx) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    ctx->timing = enable != 0;
    ctx->ktime.clear();
    ctx->spans.clear();
    if (ctx->timing) {  // the origin of the spans (qg_ctx_phase_split)
      if (!ctx->tref) QG_HIP(hipEventCreate(&ctx->tref));
      QG_HIP(hipEventRecord(ctx->tref, ctx->stream));
    }
  });
}

int qg_ctx_phase_split(const qg_ctx* ctx, const char* const* names, size_t k, double* busy_ms) {
  if (!ctx || (k && (!names || !busy_ms))) return QG_ERR_INVALID;
  std::map<std::string, size_t> idx;
  for (size_t i = 0; i < k; i++) {
    if (!names[i]) return QG_ERR_INVALID;
    idx[names[i]] = i;
    busy_ms[i] = 0.0;
  }
  // sweep over the span boundaries of the listed phases: each elementary
  // interval is shared evenly by the phases open in it
  std::vector<std::pair<double, long>> ev;  // (time, +(i+1) open / -(i+1) close)
  for (const auto& sp : ctx->spans) {
    auto it = idx.find(sp.name);
    if (it == idx.end() || !(sp.t1 > sp.t0)) continue;
    ev.push_back({sp.t0, (long)it->second + 1});
    ev.push_back({sp.t1, -((long)it->second + 1)});
  }
  std::sort(ev.begin(), ev.end());
  std::vector<int> open(k, 0);
  int nopen = 0;
  for (size_t e = 0; e < ev.size(); e++) {
    if (e > 0 && nopen > 0) {
      const double len = ev[e].first - ev[e - 1].first;
      int distinct = 0;
      for (size_t i = 0; i < k; i++) distinct += open[i] > 0;
      for (size_t i = 0; i < k; i++)
        if (open[i] > 0) busy_ms[i] += len / distinct;
    }
    const long v = ev[e].second;
    const size_t i = (size_t)(v > 0 ? v : -v) - 1;
    open[i] += v > 0 ? 1 : -1;
    nopen += v > 0 ? 1 : -1;
  }
  return QG_OK;
}

int qg_ctx_kernel_time(const qg_ctx* ctx, const char* name, double* total_ms, uint32_t* launches) {
  if (!ctx || !name) return QG_ERR_INVALID;
  auto it = ctx->ktime.find(name);
  if (total_ms) *total_ms = it == ctx->ktime.end() ? 0.0 : it->second.first;
  if (launches) *launches = it == ctx->ktime.end() ? 0 : it->second.second;
  return QG_OK;
}

int qg_ctx_counter(const qg_ctx* ctx, const char* name, uint64_t* value) {
  if (!ctx || !name || !value) return QG_ERR_INVALID;
  const std::string n(name);
  *value = n == "msm_plan_refetch"         ? ctx->msm_plan_refetch
           : n == "msm_handover_violation" ? ctx->msm_handover_violation
                                           : 0;
  return QG_OK;
}

int qg_trace_marker(qg_ctx* ctx, uint32_t tag) {
  if (!ctx || tag == 0) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    hipLaunchKernelGGL(k_trace_marker, dim3(tag), dim3(64), 0, ctx->stream);
    QG_LAUNCH_CHECK();
  });
}

// ---- transcript -----------------------------------------------------------
int qg_transcript_new(const uint8_t* domain, size_t len, uint8_t state[32]) {
  if (!state || (!domain && len)) return QG_ERR_INVALID;
  transcript_init(state, domain, len);
  return QG_OK;
}

int qg_transcript_append(uint8_t state[32], const uint8_t* msg, size_t len) {
  if (!state || (!msg && len)) return QG_ERR_INVALID;
  transcript_append(state, msg, len);
  return QG_OK;
}

int qg_transcript_draw(uint8_t state[32], uint8_t* out, size_t n) {
  if (!state || !out || n > 64) return QG_ERR_INVALID;
  transcript_draw(state, out, n);
  return QG_OK;
}

int qg_transcript_draw_fr(uint8_t state[32], uint64_t out_fr[4]) {
  if (!state || !out_fr) return QG_ERR_INVALID;
  fr_export(transcript_draw_fr(state), out_fr);
  return QG_OK;
}

int qg_fr_serialize(const uint64_t fr[4], uint8_t out[32]) {
  if (!fr || !out) return QG_ERR_INVALID;
  fr_to_bytes(fr_import(fr), out);
  return QG_OK;
}

int qg_g1_serialize(const uint64_t xy[8], uint8_t infinity, uint8_t out[64]) {
  if (!xy || !out) return QG_ERR_INVALID;
  g1_serialize(g1_import(xy, infinity), out);
  return QG_OK;
}

// ---- device vectors -------------------------------------------------------
// allocation ids of qg_buf (process-wide, never reused)
static uint64_t next_buf_id() {
  static std::atomic<uint64_t> next{0};
  return ++next;
}

int qg_buf_create(qg_ctx* ctx, size_t n, qg_buf** out) {
  if (!ctx || !out) return QG_ERR_INVALID;
  *out = nullptr;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    qg_buf* b = new qg_buf();
    b->ctx = ctx;
    b->n = n;
    b->alloc_id = next_buf_id();
    hipError_t e = hipMalloc(&b->d, (n ? n : 1) * sizeof(Fr));
    if (e != hipSuccess) {
      delete b;
      throw Error(QG_ERR_OOM, "qg_buf_create: hipMalloc failed");
    }
    *out = b;
  });
}

int qg_buf_destroy(qg_buf* buf) {
  if (!buf) return QG_OK;
  if (buf->owned) (void)hipFree(buf->d);
  delete buf;
  return QG_OK;
}

size_t qg_buf_len(const qg_buf* buf) { return buf ? buf->n : 0; }

int qg_buf_upload(qg_buf* buf, const uint64_t* fr, size_t n) {
  if (!buf || (!fr && n) || n > buf->n) return QG_ERR_INVALID;
  return qg_guard(buf->ctx, [&] {
    fr_upload(buf->ctx, buf->d, fr, n);
    buf->ctx->sync();
  });
}

int qg_buf_download(const qg_buf* buf, uint64_t* fr, size_t n) {
  if (!buf || (!fr && n) || n > buf->n) return QG_ERR_INVALID;
  return qg_guard(buf->ctx, [&] {
    fr_download(buf->ctx, fr, buf->d, n);
    buf->ctx->sync();
  });
}

int qg_buf_fill_random(qg_buf* buf, uint64_t seed) {
  if (!buf) return QG_ERR_INVALID;
  return qg_guard(buf->ctx, [&] {
    size_t blocks = (buf->n + 63) / 64;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_fill_random, dim3(div_up(blocks, 256)), dim3(256), 0, buf->ctx->stream,
                       buf->d, buf->n, seed);
    QG_LAUNCH_CHECK();
    buf->ctx->sync();
  });
}

int qg_buf_view(qg_buf* base, size_t offset, size_t n, qg_buf** out) {
  if (!base || !out || offset > base->n || n > base->n - offset) return QG_ERR_INVALID;
  *out = nullptr;
  return qg_guard(base->ctx, [&] {
    qg_buf* b = new qg_buf();
    b->ctx = base->ctx;
    b->n = n;
    b->d = base->d + offset;
    b->owned = false;
    b->alloc_id = base->alloc_id;
    b->base_off = base->base_off + offset;
    *out = b;
  });
}

int qg_buf_upload_at(qg_buf* buf, size_t offset, const uint64_t* fr, size_t n) {
  if (!buf || (!fr && n) || offset > buf->n || n > buf->n - offset) return QG_ERR_INVALID;
  return qg_guard(buf->ctx, [&] {
    fr_upload(buf->ctx, buf->d + offset, fr, n);
    buf->ctx->sync();
  });
}

int qg_buf_upload_canonical(qg_buf* buf, size_t offset, const uint64_t* canon, size_t n) {
  if (!buf || (!canon && n) || offset > buf->n || n > buf->n - offset) return QG_ERR_INVALID;
  return qg_guard(buf->ctx, [&] {
    if (n == 0) return;
    qg_ctx* ctx = buf->ctx;
    uint32_t* d_err = ctx->scratch_as<uint32_t>("canon_err", 1);
    QG_HIP(hipMemsetAsync(d_err, 0, 4, ctx->stream));
    fr_upload(ctx, buf->d + offset, canon, n);
    hipLaunchKernelGGL(k_canon_to_mont, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream,
                       buf->d + offset, n, d_err);
    QG_LAUNCH_CHECK();
    uint32_t err = 0;
    QG_HIP(hipMemcpyAsync(&err, d_err, 4, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    QG_CHECK(!err, QG_ERR_INVALID, "canonical value >= r");
  });
}

int qg_buf_upload_u64(qg_buf* buf, size_t offset, const uint64_t* v, size_t n) {
  if (!buf || (!v && n) || offset > buf->n || n > buf->n - offset) return QG_ERR_INVALID;
  return qg_guard(buf->ctx, [&] {
    if (n == 0) return;
    qg_ctx* ctx = buf->ctx;
    uint64_t* d_v = ctx->scratch_as<uint64_t>("u64_stage", n);
    QG_HIP(hipMemcpyAsync(d_v, v, n * 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_from_u64, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream,
                       buf->d + offset, d_v, n);
    QG_LAUNCH_CHECK();
    ctx->sync();
  });
}

int qg_buf_copy(qg_buf* dst, size_t dst_off, const qg_buf* src, size_t src_off, size_t n) {
  if (!dst || !src || dst_off > dst->n || n > dst->n - dst_off || src_off > src->n ||
      n > src->n - src_off)
    return QG_ERR_INVALID;
  return qg_guard(dst->ctx, [&] {
    if (n == 0) return;
    QG_HIP(hipMemcpyAsync(dst->d + dst_off, src->d + src_off, n * sizeof(Fr),
                          hipMemcpyDeviceToDevice, dst->ctx->stream));
    dst->ctx->sync();
  });
}

int qg_buf_first_mismatch(const qg_buf* a, size_t a_off, const qg_buf* b, size_t b_off, size_t n,
                          int64_t* first) {
  if (!a || !b || !first || a_off > a->n || n > a->n - a_off || b_off > b->n ||
      n > b->n - b_off)
    return QG_ERR_INVALID;
  return qg_guard(a->ctx, [&] {
    *first = -1;
    if (n == 0) return;
    qg_ctx* ctx = a->ctx;
    unsigned long long* d_f = ctx->scratch_as<unsigned long long>("mismatch", 1);
    const unsigned long long init = n;
    QG_HIP(hipMemcpyAsync(d_f, &init, 8, hipMemcpyHostToDevice, ctx->stream));
    hipLaunchKernelGGL(k_first_mismatch, dim3(div_up(n, 256)), dim3(256), 0, ctx->stream,
                       a->d + a_off, b->d + b_off, n, d_f);
    QG_LAUNCH_CHECK();
    unsigned long long f = 0;
    QG_HIP(hipMemcpyAsync(&f, d_f, 8, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
    *first = f >= n ? -1 : (int64_t)f;
  });
}

}  // extern "C"
