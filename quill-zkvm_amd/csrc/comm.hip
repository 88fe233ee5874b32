// RCCL (over xGMI) plumbing for the multi-GPU hot path.
//
// The reference has no distributed code at all; this is the
// build's own exchange layer:
//  * MSM: ranks own disjoint base/scalar shards; one allgather of the 128-byte
//    XYZZ partial per rank, then EC additions (RCCL cannot add curve points).
//  * sumcheck: ranks own the block of the hypercube selected by the high index
//    bits; one allgather of the (d+1) round sums per round.
#include <string.h>

#include <rccl/rccl.h>

#include "common.h"

struct qg_comm_state {
  ncclComm_t comm = nullptr;
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
  QG_CHECK(ctx->comm && ctx->comm->comm, QG_ERR_COMM, "no communicator attached");
  QG_NCCL(ncclAllGather(d_send, d_recv, bytes, ncclUint8, ctx->comm->comm, ctx->stream));
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
    ctx->rank = rank;
    ctx->world = world;
    if (world == 1) return;
    ncclUniqueId id;
    memcpy(&id, unique_id, 128);
    ctx->comm = new qg_comm_state();
    QG_NCCL(ncclCommInitRank(&ctx->comm->comm, world, id, rank));
  });
}

}  // extern "C"
