// warpcomm.h: one RCCL communicator per rank, collectives on the caller's
// stream (the exchange step of a row-sharded query; the reference gathers on
// the host instead, src/multi_gpu_utils.cpp:23-60).
#include "warpcomm.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>

struct wx_comm {
  ncclComm_t nc = nullptr;
  int32_t rank = 0, size = 0, device = 0;
};

namespace {

wx_status report(char *err, size_t errlen, wx_status st, const char *what, const char *detail) {
  if (err && errlen) std::snprintf(err, errlen, "%s%s%s", what, detail ? ": " : "", detail ? detail : "");
  return st;
}

wx_status nccl_status(char *err, size_t errlen, ncclResult_t r, const char *what) {
  if (r == ncclSuccess) return WX_OK;
  return report(err, errlen, WX_ERR_DEVICE, what, ncclGetErrorString(r));
}

bool nccl_type(wx_dtype t, ncclDataType_t *out) {
  switch (t) {
    case WX_INT32: *out = ncclInt32; return true;
    case WX_INT64: *out = ncclInt64; return true;
    case WX_FLOAT32: *out = ncclFloat32; return true;
    case WX_FLOAT64: *out = ncclFloat64; return true;
    default: return false;
  }
}

}  // namespace

extern "C" {

wx_status wx_comm_unique_id(unsigned char *id, char *err, size_t errlen) {
  static_assert(sizeof(ncclUniqueId) == WX_COMM_ID_BYTES, "ncclUniqueId is 128 bytes");
  if (!id) return report(err, errlen, WX_ERR_INVALID, "null id buffer", nullptr);
  ncclUniqueId u;
  const wx_status st = nccl_status(err, errlen, ncclGetUniqueId(&u), "ncclGetUniqueId");
  if (st == WX_OK) std::memcpy(id, &u, sizeof u);
  return st;
}

wx_status wx_comm_init(const unsigned char *id, int32_t n_ranks, int32_t rank, int32_t device, wx_comm **comm,
                       char *err, size_t errlen) {
  if (!id || !comm) return report(err, errlen, WX_ERR_INVALID, "null id / comm pointer", nullptr);
  if (n_ranks < 1 || rank < 0 || rank >= n_ranks) return report(err, errlen, WX_ERR_INVALID, "bad rank", nullptr);
  *comm = nullptr;
  const hipError_t he = hipSetDevice(device);
  if (he != hipSuccess) return report(err, errlen, WX_ERR_DEVICE, "hipSetDevice", hipGetErrorString(he));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof u);
  auto *c = new wx_comm;
  const wx_status st = nccl_status(err, errlen, ncclCommInitRank(&c->nc, n_ranks, u, rank), "ncclCommInitRank");
  if (st != WX_OK) {
    delete c;
    return st;
  }
  c->rank = rank;
  c->size = n_ranks;
  c->device = device;
  *comm = c;
  return WX_OK;
}

wx_status wx_comm_all_reduce(wx_comm *comm, const void *src, void *dst, int64_t count, wx_dtype dtype,
                             wx_comm_op op, void *stream, char *err, size_t errlen) {
  if (!comm || !comm->nc) return report(err, errlen, WX_ERR_INVALID, "null communicator", nullptr);
  if (count < 0 || (count > 0 && (!src || !dst))) return report(err, errlen, WX_ERR_INVALID, "bad buffer", nullptr);
  ncclDataType_t t;
  if (!nccl_type(dtype, &t)) return report(err, errlen, WX_ERR_UNSUPPORTED, "all-reduce dtype", nullptr);
  const ncclRedOp_t o = op == WX_COMM_MAX ? ncclMax : (op == WX_COMM_MIN ? ncclMin : ncclSum);
  if (count == 0) return WX_OK;
  return nccl_status(err, errlen,
                     ncclAllReduce(src, dst, (size_t)count, t, o, comm->nc, static_cast<hipStream_t>(stream)),
                     "ncclAllReduce");
}

wx_status wx_comm_all_gather(wx_comm *comm, const void *src, void *dst, int64_t bytes, void *stream, char *err,
                             size_t errlen) {
  if (!comm || !comm->nc) return report(err, errlen, WX_ERR_INVALID, "null communicator", nullptr);
  if (bytes < 0 || (bytes > 0 && (!src || !dst))) return report(err, errlen, WX_ERR_INVALID, "bad buffer", nullptr);
  if (bytes == 0) return WX_OK;
  return nccl_status(err, errlen,
                     ncclAllGather(src, dst, (size_t)bytes, ncclUint8, comm->nc, static_cast<hipStream_t>(stream)),
                     "ncclAllGather");
}

int32_t wx_comm_rank(const wx_comm *comm) { return comm ? comm->rank : -1; }
int32_t wx_comm_size(const wx_comm *comm) { return comm ? comm->size : 0; }

wx_status wx_comm_destroy(wx_comm *comm, char *err, size_t errlen) {
  if (!comm) return WX_OK;
  const wx_status st = comm->nc ? nccl_status(err, errlen, ncclCommDestroy(comm->nc), "ncclCommDestroy") : WX_OK;
  delete comm;
  return st;
}

}  // extern "C"
