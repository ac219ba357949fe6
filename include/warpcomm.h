/*
 * warpcomm.h -- the exchange step of a row-sharded query: one RCCL
 * communicator per rank (one process per GPU), its collectives enqueued on
 * the query's own stream.
 *
 * Reference interface replaced: the multi-GPU loop of run_multi_gpu_jit_host
 * (src/multi_gpu_utils.cpp:23-60), which copies every shard's dense result to
 * the host and concatenates there.  Here the shards' partials meet in HBM
 * through one RCCL collective (xGMI) and are merged by a warpexec kernel
 * (wx_group_combine_slots, wx_topk_merge, wx_head_merge, ...).
 *
 * Why a communicator of its own beside torch.distributed's: a
 * torch.distributed collective runs on that process group's internal stream,
 * so every exchange costs two cross-stream event waits (the collective after
 * the partials kernel, the merge kernel after the collective) -- about 14 us
 * of a 160-us GROUP BY step at the 8-GPU per-rank size.  These calls enqueue
 * ncclAllReduce / ncclAllGather on the stream the kernels run on: stream order
 * is the only synchronisation.  (The single-process multi-GPU engine,
 * ResidentShards in libwarpdb, does the same with ncclCommInitAll.)
 *
 * Usage (every rank): rank 0 calls wx_comm_unique_id and hands the 128 bytes
 * to the others (torch.distributed broadcast, a file, ...); every rank then
 * calls wx_comm_init with the same id -- a collective call that returns once
 * all n_ranks have joined.  Implemented in libwarpdb.so.
 */
#ifndef WARPCOMM_H
#define WARPCOMM_H

#include "warpexec.h"

#ifdef __cplusplus
extern "C" {
#endif

#define WX_COMM_ID_BYTES 128

typedef struct wx_comm wx_comm;

typedef enum wx_comm_op { WX_COMM_SUM = 0, WX_COMM_MAX = 1, WX_COMM_MIN = 2 } wx_comm_op;

/* A fresh communicator id (ncclGetUniqueId), on rank 0. */
wx_status wx_comm_unique_id(unsigned char *id /* WX_COMM_ID_BYTES */, char *err, size_t errlen);

/* This rank's communicator on `device` (ncclCommInitRank; blocks until every
 * rank has called it with the same id). */
wx_status wx_comm_init(const unsigned char *id, int32_t n_ranks, int32_t rank, int32_t device, wx_comm **comm,
                       char *err, size_t errlen);

/* count elements of dtype (WX_INT32, WX_INT64, WX_FLOAT32, WX_FLOAT64),
 * reduced over the ranks into dst (dst == src: in place), on `stream`. */
wx_status wx_comm_all_reduce(wx_comm *comm, const void *src, void *dst, int64_t count, wx_dtype dtype,
                             wx_comm_op op, void *stream, char *err, size_t errlen);

/* `bytes` from every rank, concatenated in rank order into dst (n_ranks x
 * bytes), on `stream`. */
wx_status wx_comm_all_gather(wx_comm *comm, const void *src, void *dst, int64_t bytes, void *stream, char *err,
                             size_t errlen);

/* Rank and size of the communicator. */
int32_t wx_comm_rank(const wx_comm *comm);
int32_t wx_comm_size(const wx_comm *comm);

/* Releases the communicator (ncclCommDestroy); NULL is a no-op. */
wx_status wx_comm_destroy(wx_comm *comm, char *err, size_t errlen);

#ifdef __cplusplus
}
#endif

#endif /* WARPCOMM_H */
