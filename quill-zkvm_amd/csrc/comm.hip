// RCCL (over xGMI) plumbing for the multi-GPU hot path.
//
// The reference has no distributed code at all; this is the
// build's own exchange layer:
//  * MSM: ranks own disjoint base/scalar shards; one allgather of the 128-byte
//    XYZZ partial per rank, then EC additions (RCCL cannot add curve points).
//  * sumcheck: ranks own the block of the hypercube selected by the high index
//    bits; one allgather of the (d+1) round sums per round.
//  * ML-PCS opening: the S polynomial's transform is split by frequency
//    residue; one all-to-all delivers every rank its slice of S.
#include <stdlib.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

#include <algorithm>
#include <vector>

#include "common.h"

// In-process loopback group: `world` contexts driven by `world` host threads
// on one device.  Same collective hook as RCCL; used to exercise every sharded
// code path on a single GPU (tests/test_gpu_multirank.py).
struct qg_loopback {
  int world = 0;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> sends;

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      generation++;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};

struct qg_comm_state {
  ncclComm_t comm = nullptr;
  qg_loopback* lb = nullptr;
};

namespace qg {

#define QG_NCCL(call)                                                                  \
  do {                                                                                 \
    ncclResult_t _r = (call);                                                          \
    if (_r != ncclSuccess)                                                             \
      throw ::qg::Error(QG_ERR_COMM, std::string(#call) + ": " + ncclGetErrorString(_r)); \
  } while (0)

void comm_allgather_bytes(qg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes) {
  if (!ctx->sharded) {
    QG_HIP(hipMemcpyAsync(d_recv, d_send, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return;
  }
  QG_CHECK(ctx->comm, QG_ERR_COMM, "no communicator attached");
  if (ctx->comm->lb) {
    qg_loopback* lb = ctx->comm->lb;
    QG_HIP(hipStreamSynchronize(ctx->stream));  // send buffer complete
    lb->sends[ctx->rank] = d_send;
    lb->barrier();
    for (int r = 0; r < ctx->world; r++)
      QG_HIP(hipMemcpyAsync((uint8_t*)d_recv + (size_t)r * bytes, lb->sends[r], bytes,
                            hipMemcpyDeviceToDevice, ctx->stream));
    QG_HIP(hipStreamSynchronize(ctx->stream));
    lb->barrier();  // nobody reuses its send buffer before every rank has copied it
    return;
  }
  QG_CHECK(ctx->comm->comm, QG_ERR_COMM, "no communicator attached");
  QG_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, ctx->comm->comm, ctx->stream));
}

// Personalised exchange: d_send holds world chunks of `bytes` (chunk d goes to
// rank d), d_recv receives world chunks (chunk s came from rank s).  RCCL:
// grouped point-to-point send/recv over xGMI (no reduction: the payload is
// field elements, which RCCL cannot add); loopback: device copies.
void comm_alltoall_bytes(qg_ctx* ctx, const void* d_send, void* d_recv, size_t bytes) {
  if (!ctx->sharded) {
    QG_HIP(hipMemcpyAsync(d_recv, d_send, bytes, hipMemcpyDeviceToDevice, ctx->stream));
    return;
  }
  QG_CHECK(ctx->comm, QG_ERR_COMM, "no communicator attached");
  if (ctx->comm->lb) {
    qg_loopback* lb = ctx->comm->lb;
    QG_HIP(hipStreamSynchronize(ctx->stream));  // send buffer complete
    lb->sends[ctx->rank] = d_send;
    lb->barrier();
    for (int r = 0; r < ctx->world; r++)
      QG_HIP(hipMemcpyAsync((uint8_t*)d_recv + (size_t)r * bytes,
                            (const uint8_t*)lb->sends[r] + (size_t)ctx->rank * bytes, bytes,
                            hipMemcpyDeviceToDevice, ctx->stream));
    QG_HIP(hipStreamSynchronize(ctx->stream));
    lb->barrier();
    return;
  }
  QG_CHECK(ctx->comm->comm, QG_ERR_COMM, "no communicator attached");
  QG_NCCL(ncclGroupStart());
  for (int r = 0; r < ctx->world; r++) {
    QG_NCCL(ncclSend((const uint8_t*)d_send + (size_t)r * bytes, bytes, ncclUint8, r,
                     ctx->comm->comm, ctx->stream));
    QG_NCCL(ncclRecv((uint8_t*)d_recv + (size_t)r * bytes, bytes, ncclUint8, r, ctx->comm->comm,
                     ctx->stream));
  }
  QG_NCCL(ncclGroupEnd());
}

// One contiguous piece of a sharded column-major full witness: rows [a, b) of
// column c travel from rank `src` (its row block of c) to rank `dst` (its block
// of the flattened trace).
struct TraceChunk {
  uint32_t c, src, dst;
  size_t a, b;
};

static std::vector<TraceChunk> trace_chunks(uint32_t ncols, size_t rows, int world) {
  std::vector<TraceChunk> out;
  const size_t RL = rows / world, B = (size_t)ncols * rows / world;
  for (uint32_t c = 0; c < ncols; c++)
    for (int src = 0; src < world; src++) {
      size_t a = src * RL;
      const size_t end = a + RL;
      while (a < end) {  // split the source rows at destination-block boundaries
        const size_t flat = (size_t)c * rows + a;
        const uint32_t dst = (uint32_t)(flat / B);
        const size_t dst_end_row = ((size_t)(dst + 1) * B) - (size_t)c * rows;
        const size_t b = std::min(end, dst_end_row);
        out.push_back({c, (uint32_t)src, dst, a, b});
        a = b;
      }
    }
  return out;
}

// full_block = this rank's block of concat(columns) (hyperplonk/src/proof/proof.rs:270),
// from every rank's row block of each column
void trace_full_witness(qg_ctx* ctx, const std::vector<const Fr*>& cols, size_t rows, Fr* full) {
  const uint32_t ncols = (uint32_t)cols.size();
  const int world = ctx->world, rank = ctx->rank;
  if (!ctx->sharded) {
    for (uint32_t c = 0; c < ncols; c++)
      QG_HIP(hipMemcpyAsync(full + (size_t)c * rows, cols[c], rows * sizeof(Fr),
                            hipMemcpyDeviceToDevice, ctx->stream));
    ctx->sync();
    return;
  }
  QG_CHECK(ctx->comm, QG_ERR_COMM, "no communicator attached");
  const size_t RL = rows / world, B = (size_t)ncols * rows / world;
  // One allgather of every rank's packed row blocks (the collective the MSM
  // already uses), then each rank copies out its block of the flattening.  The
  // exchange moves the whole trace to every rank (N x the data of an
  // all-to-all) but is a few ms next to the proof, over one well-trodden path.
  const size_t per = (size_t)ncols * RL;
  Fr* pack = ctx->scratch_as<Fr>("tw_pack", per);
  Fr* all = ctx->scratch_as<Fr>("tw_all", per * world);
  for (uint32_t c = 0; c < ncols; c++)
    QG_HIP(hipMemcpyAsync(pack + (size_t)c * RL, cols[c], RL * sizeof(Fr), hipMemcpyDeviceToDevice,
                          ctx->stream));
  comm_allgather_bytes(ctx, pack, all, per * sizeof(Fr));
  for (const TraceChunk& k : trace_chunks(ncols, rows, world)) {
    if ((int)k.dst != rank) continue;
    const Fr* src = all + (size_t)k.src * per + (size_t)k.c * RL + (k.a - (size_t)k.src * RL);
    QG_HIP(hipMemcpyAsync(full + ((size_t)k.c * rows + k.a - (size_t)rank * B), src,
                          (k.b - k.a) * sizeof(Fr), hipMemcpyDeviceToDevice, ctx->stream));
  }
  ctx->sync();
}

bool comm_is_loopback(const qg_ctx* ctx) { return ctx->comm && ctx->comm->lb; }

void comm_release(qg_ctx* ctx) {
  if (!ctx->comm) return;
  if (ctx->comm->comm) (void)ncclCommDestroy(ctx->comm->comm);
  delete ctx->comm;  // a loopback group is owned by its creator
  ctx->comm = nullptr;
  ctx->sharded = false;
}

bool comm_is_rccl(const qg_ctx* ctx) { return ctx->comm && ctx->comm->comm; }

}  // namespace qg

using namespace qg;

extern "C" {

int qg_comm_unique_id(uint8_t out_id[128]) {
  if (!out_id) return QG_ERR_INVALID;
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return QG_ERR_COMM;
  static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
  memcpy(out_id, &id, 128);
  return QG_OK;
}

int qg_ctx_attach_comm(qg_ctx* ctx, int rank, int world, const uint8_t unique_id[128]) {
  if (!ctx || world < 1 || rank < 0 || rank >= world || (!unique_id && world > 1))
    return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    if (ctx->comm) {
      if (ctx->comm->comm) (void)ncclCommDestroy(ctx->comm->comm);
      delete ctx->comm;
      ctx->comm = nullptr;
    }
    ctx->rank = 0;
    ctx->world = 1;
    ctx->sharded = false;
    // QG_FORCE_RCCL=1 (test switch): a world-1 context still attaches a real
    // one-rank RCCL communicator and takes the sharded paths, so a 1-GPU box
    // executes ncclCommInitRank / ncclAllGather / grouped ncclSend+ncclRecv
    const char* force = getenv("QG_FORCE_RCCL");
    const bool forced = world == 1 && force && force[0] && strcmp(force, "0") != 0;
    if (world == 1 && !forced) return;
    ncclUniqueId id;
    if (unique_id)
      memcpy(&id, unique_id, 128);
    else
      QG_NCCL(ncclGetUniqueId(&id));
    ctx->comm = new qg_comm_state();
    QG_NCCL(ncclCommInitRank(&ctx->comm->comm, world, id, rank));
    ctx->rank = rank;
    ctx->world = world;
    ctx->sharded = true;
  });
}

int qg_comm_allgather_host(qg_ctx* ctx, const void* send, size_t bytes, void* recv) {
  if (!ctx || (!send && bytes) || (!recv && bytes)) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    if (bytes == 0) return;
    QG_HIP(hipSetDevice(ctx->device));
    uint8_t* d = ctx->scratch_as<uint8_t>("ag_host", bytes * (size_t)(ctx->world + 1));
    QG_HIP(hipMemcpyAsync(d, send, bytes, hipMemcpyHostToDevice, ctx->stream));
    comm_allgather_bytes(ctx, d, d + bytes, bytes);
    QG_HIP(hipMemcpyAsync(recv, d + bytes, bytes * (size_t)ctx->world, hipMemcpyDeviceToHost,
                          ctx->stream));
    ctx->sync();
  });
}

int qg_comm_alltoall_host(qg_ctx* ctx, const void* send, size_t bytes, void* recv) {
  if (!ctx || (!send && bytes) || (!recv && bytes)) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    if (bytes == 0) return;
    QG_HIP(hipSetDevice(ctx->device));
    const size_t all = bytes * (size_t)ctx->world;
    uint8_t* d = ctx->scratch_as<uint8_t>("a2a_host", 2 * all);
    QG_HIP(hipMemcpyAsync(d, send, all, hipMemcpyHostToDevice, ctx->stream));
    comm_alltoall_bytes(ctx, d, d + all, bytes);
    QG_HIP(hipMemcpyAsync(recv, d + all, all, hipMemcpyDeviceToHost, ctx->stream));
    ctx->sync();
  });
}

int qg_ctx_comm_info(const qg_ctx* ctx, int* kind, int* rank, int* world, int* sharded) {
  if (!ctx) return QG_ERR_INVALID;
  if (kind) *kind = !ctx->comm ? 0 : ctx->comm->lb ? 1 : ctx->comm->comm ? 2 : 0;
  if (rank) *rank = ctx->rank;
  if (world) *world = ctx->world;
  if (sharded) *sharded = ctx->sharded ? 1 : 0;
  return QG_OK;
}

int qg_trace_full_witness(qg_ctx* ctx, const qg_buf* const* col_blocks, uint32_t ncols,
                          uint64_t rows, qg_buf* full_block) {
  if (!ctx || !col_blocks || !ncols || !full_block) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    QG_HIP(hipSetDevice(ctx->device));
    const int world = ctx->world;
    QG_CHECK(rows % world == 0 && ((size_t)ncols * rows) % world == 0, QG_ERR_INVALID,
             "rows and cells must divide by the world size");
    const size_t RL = rows / world, B = (size_t)ncols * rows / world;
    QG_CHECK(full_block->n >= B, QG_ERR_INVALID, "full-witness block too short");
    std::vector<const Fr*> cols;
    for (uint32_t c = 0; c < ncols; c++) {
      QG_CHECK(col_blocks[c] && col_blocks[c]->n >= RL, QG_ERR_INVALID,
               "column block missing or too short");
      QG_CHECK(col_blocks[c]->d + RL <= full_block->d || full_block->d + B <= col_blocks[c]->d,
               QG_ERR_INVALID, "full witness aliases a column block");
      cols.push_back(col_blocks[c]->d);
    }
    trace_full_witness(ctx, cols, rows, full_block->d);
  });
}

int qg_loopback_create(int world, qg_loopback** out) {
  if (!out || world < 1) return QG_ERR_INVALID;
  qg_loopback* lb = new qg_loopback();
  lb->world = world;
  lb->sends.assign(world, nullptr);
  *out = lb;
  return QG_OK;
}

int qg_loopback_destroy(qg_loopback* lb) {
  delete lb;
  return QG_OK;
}

int qg_ctx_attach_loopback(qg_ctx* ctx, qg_loopback* lb, int rank) {
  if (!ctx || !lb || rank < 0 || rank >= lb->world) return QG_ERR_INVALID;
  return qg_guard(ctx, [&] {
    if (ctx->comm) {
      if (ctx->comm->comm) (void)ncclCommDestroy(ctx->comm->comm);
      delete ctx->comm;
    }
    ctx->comm = new qg_comm_state();
    ctx->comm->lb = lb;
    ctx->rank = rank;
    ctx->world = lb->world;
    ctx->sharded = true;  // a one-rank group too: the sharded paths at world 1
  });
}

}  // extern "C"
