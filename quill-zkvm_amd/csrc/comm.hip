// RCCL (over xGMI) plumbing for the multi-GPU hot path.
//
// The reference has no distributed code at all; this is the
// build's own exchange layer:
//  * MSM: ranks own disjoint base/scalar shards; one allgather of the 128-byte
//    XYZZ partial per rank, then EC additions (RCCL cannot add curve points).
//  * sumcheck: ranks own the block of the hypercube selected by the high index
//    bits; one allgather of the (d+1) round sums per round.
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <vector>

#include <rccl/rccl.h>

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
  if (ctx->world <= 1) {
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

void comm_release(qg_ctx* ctx) {
  if (!ctx->comm) return;
  if (ctx->comm->comm) (void)ncclCommDestroy(ctx->comm->comm);
  delete ctx->comm;  // a loopback group is owned by its creator
  ctx->comm = nullptr;
}

}  // namespace qg

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
    ctx->rank = rank;
    ctx->world = world;
    if (world == 1) return;
    ncclUniqueId id;
    memcpy(&id, unique_id, 128);
    ctx->comm = new qg_comm_state();
    QG_NCCL(ncclCommInitRank(&ctx->comm->comm, world, id, rank));
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
  });
}

}  // extern "C"
