// Shared host-side infrastructure of libquill_gpu: context, scratch arena,
// error handling at the C-ABI, HIP-event kernel timing.
#pragma once
#include <hip/hip_runtime.h>

#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/quill_gpu.h"
#include "arena.h"
#include "curve.h"
#include "field.h"

namespace qg {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define QG_HIP(call)                                                                  \
  do {                                                                                \
    hipError_t _e = (call);                                                           \
    if (_e != hipSuccess)                                                             \
      throw ::qg::Error(_e == hipErrorOutOfMemory ? QG_ERR_OOM : QG_ERR_DEVICE,       \
                        std::string(#call) + ": " + hipGetErrorString(_e));           \
  } while (0)

#define QG_CHECK(cond, code, msg)                  \
  do {                                             \
    if (!(cond)) throw ::qg::Error((code), (msg)); \
  } while (0)

// Launch-and-check helper: kernel errors surface at the call.
#define QG_LAUNCH_CHECK() QG_HIP(hipGetLastError())

inline unsigned div_up(size_t a, size_t b) { return (unsigned)((a + b - 1) / b); }

// device-memory backend of the scratch arena (arena.h)
struct HipAlloc {
  // a slot that grows is released while kernels queued on the context's
  // streams (the MSM batch's side streams included) may still read it: the
  // owning context drains exactly those streams (not the device: loopback
  // ranks share it), and a failure surfaces as an error
  void (*drain)(void* owner) = nullptr;
  void* owner = nullptr;
  static void* alloc(size_t b) {
    void* p = nullptr;
    QG_HIP(hipMalloc(&p, b));
    return p;
  }
  void release(void* p) {
    if (drain)
      drain(owner);
    else
      QG_HIP(hipDeviceSynchronize());
    QG_HIP(hipFree(p));
  }
};

}  // namespace qg

struct qg_comm_state;  // RCCL (comm.hip)

struct qg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // host-to-device uploads overlapped with kernels (msm_host)
  hipStream_t side_stream = nullptr;   // MSM batches on two side streams, by MSM parity
  hipStream_t side_stream2 = nullptr;  // (QG_MSM_PIPE=1, msm.hip)
  std::string last_error;
  // grow-only scratch arena, one slot per purpose; every (re)allocation and
  // every table build gets a fresh generation number (arena.h), which caches
  // key on instead of device addresses
  qg::ScratchArena<qg::HipAlloc> arena;  // backend.drain = drain_streams (qg_ctx_create)
  qg::LruSlots<4> twm_lru;  // S polynomial: w^{j(M-1)} tables per (logn, M)
  // timing
  bool timing = false;
  struct Ev {
    std::string name;
    hipEvent_t a, b;
    bool ended;
    hipStream_t s;
  };
  std::map<int, Ev> pending;  // handle -> region (stable across nested syncs)
  int next_handle = 0;
  std::map<std::string, std::pair<double, uint32_t>> ktime;
  // every resolved region as [t0, t1) ms after the timing origin `tref`
  // (recorded on the context stream when timing is enabled): the additive
  // busy-time split of qg_ctx_phase_split
  hipEvent_t tref = nullptr;
  struct Span {
    std::string name;
    float t0, t1;
  };
  std::vector<Span> spans;
  std::vector<hipEvent_t> event_pool;
  // small per-context memo (e.g. which program image the device copy holds)
  std::map<std::string, std::string> memo;
  // RCCL
  qg_comm_state* comm = nullptr;
  int rank = 0, world = 1;
  // the sharded code paths run (and exchange through the communicator): world > 1,
  // or a one-rank group (a world-1 loopback, or the one-rank RCCL communicator
  // QG_FORCE_RCCL=1 attaches so a 1-GPU box executes the RCCL transport)
  bool sharded = false;
  // MSM bucket-scan plan copies: generation tag of the last run, and the number
  // of copies found stale (re-read synchronously; stays 0 when the event
  // ordering holds)
  uint32_t msm_gen = 0;
  uint64_t msm_plan_refetch = 0;
  // MSM batches whose event-ordered cross-stream hand-over the device guard
  // found unordered (recomputed in stream order; msm.hip, msm_device_batch)
  uint64_t msm_handover_violation = 0;
  // trim_launch's call generation (mlpcs.hip: the tail launch's stamp)
  uint64_t trim_gen = 0;

  // every stream of this context, synchronized (scratch release, destroy)
  static void drain_streams(void* self) {
    qg_ctx* c = static_cast<qg_ctx*>(self);
    for (hipStream_t s : {c->stream, c->copy_stream, c->side_stream, c->side_stream2})
      if (s) QG_HIP(hipStreamSynchronize(s));
  }

  int cus = 0;  // compute units of `device` (cached)
  int num_cus() {
    if (!cus) QG_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    return cus;
  }

  void* scratch_get(const std::string& slot, size_t bytes) { return arena.get(slot, bytes); }
  uint64_t scratch_gen(const std::string& slot) const { return arena.gen(slot); }
  template <class T>
  T* scratch_as(const std::string& slot, size_t count) {
    return reinterpret_cast<T*>(scratch_get(slot, count * sizeof(T)));
  }
  // grow-only pinned host staging (small per-call transfers: no pageable bounce)
  std::map<std::string, std::pair<void*, size_t>> pinned;
  void* pinned_get(const std::string& slot, size_t bytes) {
    auto it = pinned.find(slot);
    if (it != pinned.end() && it->second.second >= bytes) return it->second.first;
    if (it != pinned.end()) {
      QG_HIP(hipHostFree(it->second.first));
      pinned.erase(it);
    }
    void* p = nullptr;
    size_t b = bytes ? bytes : 16;
    QG_HIP(hipHostMalloc(&p, b, hipHostMallocDefault));
    pinned[slot] = {p, b};
    return p;
  }

  hipEvent_t ev_get() {
    if (!event_pool.empty()) {
      hipEvent_t e = event_pool.back();
      event_pool.pop_back();
      return e;
    }
    hipEvent_t e;
    QG_HIP(hipEventCreate(&e));
    return e;
  }
  // begin/end a timed region on the context stream (or on stream s)
  int tbegin(const char* name, hipStream_t s = nullptr) {
    if (!timing) return -1;
    Ev e{name, ev_get(), ev_get(), false, s ? s : stream};
    QG_HIP(hipEventRecord(e.a, e.s));
    const int h = next_handle++;
    pending[h] = e;
    return h;
  }
  void tend(int h) noexcept {
    auto it = pending.find(h);
    if (h < 0 || it == pending.end()) return;
    (void)hipEventRecord(it->second.b, it->second.s);
    it->second.ended = true;
  }
  // resolve the closed regions (after a stream sync); open ones stay pending
  void tresolve() {
    for (auto it = pending.begin(); it != pending.end();) {
      if (!it->second.ended) {
        ++it;
        continue;
      }
      float ms = 0.f;
      QG_HIP(hipEventElapsedTime(&ms, it->second.a, it->second.b));
      auto& slot = ktime[it->second.name];
      slot.first += ms;
      slot.second += 1;
      if (tref) {
        float t0 = 0.f;
        QG_HIP(hipEventElapsedTime(&t0, tref, it->second.a));
        spans.push_back({it->second.name, t0, t0 + ms});
      }
      event_pool.push_back(it->second.a);
      event_pool.push_back(it->second.b);
      it = pending.erase(it);
    }
  }
  void sync() {
    QG_HIP(hipStreamSynchronize(stream));
    if (timing) tresolve();
  }
};

struct qg_buf {
  qg_ctx* ctx = nullptr;
  size_t n = 0;
  qg::Fr* d = nullptr;
  bool owned = true;  // false: a view into another buffer (qg_buf_view)
  // identity of the allocation behind d (never reused, unlike the address) and
  // d's offset in it: what transform caches key on (s_poly_device's F)
  uint64_t alloc_id = 0;
  size_t base_off = 0;
};

struct qg_srs {
  qg_ctx* ctx = nullptr;
  size_t n = 0;  // number of bases
  int c = 0;     // MSM window bits (signed digits)
  int W = 0;     // number of windows = ceil(255 / c)
  // tables * n rows; table[w * n + i] = 2^(c*w) * base_i   (curve.h MsmPt layout)
  // tables == W: window-shifted tables (a fixed SRS); tables == 1: bases for
  // one-shot MSMs (qg_bases_upload), whose windows are summed by Horner steps
  int tables = 0;
  qg::MsmPt* d_table = nullptr;
};

// scoped timer
struct QgTimed {
  qg_ctx* c;
  int h;
  QgTimed(qg_ctx* ctx, const char* name, hipStream_t s = nullptr) : c(ctx), h(ctx->tbegin(name, s)) {}
  ~QgTimed() { c->tend(h); }
};

// Wrap a C-ABI body: no exception crosses the boundary.
template <class F>
static int qg_guard(qg_ctx* ctx, F&& f) {
  try {
    f();
    return QG_OK;
  } catch (const qg::Error& e) {
    if (ctx) ctx->last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    if (ctx) ctx->last_error = "host allocation failed";
    return QG_ERR_OOM;
  } catch (const std::exception& e) {
    if (ctx) ctx->last_error = e.what();
    return QG_ERR_DEVICE;
  } catch (...) {
    if (ctx) ctx->last_error = "unknown error";
    return QG_ERR_DEVICE;
  }
}

// ---- internal entry points shared between translation units -------------
namespace qg {
// MSM over device scalars; result (XYZZ, summed over RCCL ranks if attached)
G1Affine msm_device(qg_ctx* ctx, const qg_srs* srs, const Fr* d_scalars, size_t n);
// k MSMs over one SRS with shared reduction launches (null scalars allowed when n = 0)
std::vector<G1Affine> msm_device_batch(qg_ctx* ctx, const qg_srs* srs,
                                       const std::vector<const Fr*>& scalars,
                                       const std::vector<size_t>& ns);
void fr_upload(qg_ctx* ctx, Fr* d, const uint64_t* h, size_t n);
void fr_download(qg_ctx* ctx, uint64_t* h, const Fr* d, size_t n);
// affine G1 -> ABI (xy Montgomery limbs + inf flag)
void g1_export(const G1Affine& a, uint64_t xy[8], uint8_t* inf);
G1Affine g1_import(const uint64_t xy[8], uint8_t inf);
void g1_serialize(const G1Affine& a, uint8_t out[64]);
Fr fr_import(const uint64_t v[4]);
void fr_export(const Fr& a, uint64_t v[4]);
// eq(bin(i), z) table on the device (sumcheck.hip)
void eq_table_device(qg_ctx* ctx, const Fr* d_z, uint32_t nvars, Fr* d_out);
// h(x) per row by the generic expression interpreter (sumcheck.hip)
void expr_table_device(qg_ctx* ctx, size_t n, uint32_t ntables, const std::vector<const Fr*>& tabs,
                       const qg_expr_op* prog, size_t prog_len, const uint64_t* consts,
                       size_t nconsts, Fr* d_out);
// RCCL helpers (comm.hip); no-ops when world == 1
void comm_allgather_bytes(qg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes);
void comm_alltoall_bytes(qg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes);
void comm_release(qg_ctx* ctx);
// true when the attached communicator is the in-process loopback (ranks share a device)
bool comm_is_loopback(const qg_ctx* ctx);
}  // namespace qg
