/* surfhip_comm.h -- the multi-GPU exchange of the MI355X SURF engine
 * (libsurfcomm.so): one RCCL communicator per process/GPU and ONE
 * all-gather of fixed-capacity result slabs per batch.
 *
 * The reference is single-GPU (cuda_utils.h:41-67, no collectives); this is
 * the exchange north_star adds: frames shard as contiguous ranges over the
 * GPUs of a node, every rank runs detect+describe on its own frames
 * (surfhip_detect_batch), packs its result slab into a buffer of a capacity
 * agreed once (surfhip_pack_slab_cap: no host sync per batch) and the slabs
 * are all-gathered over xGMI, rank r's at offset r * slab_cap.
 *
 * Plain C: pointers, sizes, int status (SURFHIP_OK / SURFHIP_ERR_*).
 * A C++ caller (the reference's only kind) drives it as:
 *   rank 0: surfhip_comm_unique_id(id); share the 128 bytes out of band
 *   every rank: surfhip_set_device(local); surfhip_comm_init(&c, n, r, id);
 *   per batch: surfhip_detect_batch(...); surfhip_pack_slab_cap(..., send, cap);
 *              surfhip_allgather(c, send, cap, recv, stream);
 * (INTEGRATION.md shows it end to end). */
#pragma once

#include <stddef.h>

#include "surfhip.h"

#ifdef __cplusplus
extern "C" {
#endif

#define SURFHIP_COMM_ID_BYTES 128

typedef struct surfhip_comm surfhip_comm;

/* ncclGetUniqueId: call on one rank, pass the bytes to every rank. */
int surfhip_comm_unique_id(void* id);
/* ncclCommInitRank on the current device (blocks until all ranks joined). */
int surfhip_comm_init(surfhip_comm** out, int nranks, int rank, const void* id);
int surfhip_comm_destroy(surfhip_comm* comm);
int surfhip_comm_rank(surfhip_comm* comm, int* rank, int* nranks);
/* All-gather of `bytes` from d_send on every rank into d_recv
 * (nranks * bytes), rank r's bytes at d_recv + r * bytes; asynchronous on
 * `stream` (NULL = the null stream).  d_send may alias d_recv + rank*bytes. */
int surfhip_allgather(surfhip_comm* comm, const void* d_send, size_t bytes, void* d_recv, void* stream);
/* Sum-reduce of n int64 values (e.g. keypoint totals), in place, async. */
int surfhip_allreduce_sum_i64(surfhip_comm* comm, long long* d_vals, int n, void* stream);
/* The RCCL error of the last failing call in this thread (ncclResult_t). */
int surfhip_comm_last_error(void);

#ifdef __cplusplus
}
#endif
