// comm.hip — the data-parallel gradient exchange as C-ABI entry points over RCCL (xGMI).
//
// The reference's only collective is the implicit DDP all-reduce (sum / world) of every trainable
// gradient inside accelerate (src/train.py:61-64, src/trainer/base.py:150).  The Python host runs
// it through torch.distributed (vspike/dp.py); these entry points give a non-Python host the same
// exchange: one communicator per process / GPU, and an in-place sum all-reduce of one gradient
// bucket enqueued on the caller's stream (so it orders after the backward kernels that produced
// the bucket and before the optimizer step, and overlaps whatever the caller runs on other
// streams).  The 1/world scale is folded into the optimizer (vs_adamw grad_scale), as in dp.py.
#include <rccl/rccl.h>
#include <string.h>

#include "common.h"

static_assert(sizeof(ncclUniqueId) <= VS_COMM_ID_BYTES, "VS_COMM_ID_BYTES too small for ncclUniqueId");

namespace vs {
static int nccl_rc(ncclResult_t r, const char* what) {
  if (r == ncclSuccess) return VS_OK;
  set_error(what);
  return VS_COMM_ERR_BASE + (int)r;
}
}  // namespace vs

extern "C" int vs_comm_unique_id(void* id_out) {
  VS_REQUIRE(id_out, "vs_comm_unique_id: null id");
  ncclUniqueId id;
  memset(&id, 0, sizeof(id));
  const int rc = vs::nccl_rc(ncclGetUniqueId(&id), "vs_comm_unique_id: ncclGetUniqueId failed");
  if (rc != VS_OK) return rc;
  memset(id_out, 0, VS_COMM_ID_BYTES);
  memcpy(id_out, &id, sizeof(id));
  return VS_OK;
}

extern "C" int vs_comm_init(void** comm, const void* id, int32_t world, int32_t rank) {
  VS_REQUIRE(comm && id, "vs_comm_init: null argument");
  VS_REQUIRE(world >= 1 && rank >= 0 && rank < world, "vs_comm_init: bad world / rank");
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const int rc = vs::nccl_rc(ncclCommInitRank(&c, world, uid, rank), "vs_comm_init: ncclCommInitRank failed");
  if (rc != VS_OK) return rc;
  *comm = (void*)c;
  return VS_OK;
}

extern "C" int vs_comm_allreduce_bucket(void* comm, void* buf, int64_t count, int32_t dtype, void* stream) {
  VS_REQUIRE(comm, "vs_comm_allreduce_bucket: null communicator");
  VS_REQUIRE(count >= 0, "vs_comm_allreduce_bucket: negative count");
  VS_REQUIRE(dtype == VS_F32 || dtype == VS_BF16, "vs_comm_allreduce_bucket: dtype must be VS_F32 or VS_BF16");
  if (count == 0) return VS_OK;
  VS_REQUIRE(buf, "vs_comm_allreduce_bucket: null buffer");
  return vs::nccl_rc(ncclAllReduce(buf, buf, (size_t)count, dtype == VS_F32 ? ncclFloat32 : ncclBfloat16, ncclSum,
                                   (ncclComm_t)comm, (hipStream_t)stream),
                     "vs_comm_allreduce_bucket: ncclAllReduce failed");
}

extern "C" int vs_comm_finalize(void* comm) {
  if (!comm) return VS_OK;
  return vs::nccl_rc(ncclCommDestroy((ncclComm_t)comm), "vs_comm_finalize: ncclCommDestroy failed");
}
