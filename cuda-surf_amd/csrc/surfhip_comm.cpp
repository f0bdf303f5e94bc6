// surfhip_comm.cpp -- libsurfcomm.so: the C-ABI multi-GPU exchange
// (include/surfhip_comm.h) over RCCL.  One communicator per process/GPU,
// ncclAllGather of fixed-capacity result slabs.  Kept out of
// libsurfhip so that single-GPU users do not depend on RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <new>

#include "surfhip_comm.h"

static thread_local ncclResult_t g_last_nccl = ncclSuccess;

#define NCCLCHK(x)                       \
    do {                                 \
        ncclResult_t r_ = (x);           \
        if (r_ != ncclSuccess) {         \
            g_last_nccl = r_;            \
            return SURFHIP_ERR_HIP;      \
        }                                \
    } while (0)

struct surfhip_comm {
    ncclComm_t nc = nullptr;
    int rank = 0, nranks = 1;
};

static_assert(sizeof(ncclUniqueId) == SURFHIP_COMM_ID_BYTES, "ncclUniqueId size");

extern "C" {

int surfhip_comm_unique_id(void* id)
{
    if (!id) return SURFHIP_ERR_INVALID;
    ncclUniqueId u;
    NCCLCHK(ncclGetUniqueId(&u));
    __builtin_memcpy(id, &u, sizeof u);
    return SURFHIP_OK;
}

int surfhip_comm_init(surfhip_comm** out, int nranks, int rank, const void* id)
{
    if (!out || !id || nranks < 1 || rank < 0 || rank >= nranks) return SURFHIP_ERR_INVALID;
    ncclUniqueId u;
    __builtin_memcpy(&u, id, sizeof u);
    surfhip_comm* c = new (std::nothrow) surfhip_comm;
    if (!c) return SURFHIP_ERR_NOMEM;
    const ncclResult_t r = ncclCommInitRank(&c->nc, nranks, u, rank);
    if (r != ncclSuccess) {
        g_last_nccl = r;
        delete c;
        return SURFHIP_ERR_HIP;
    }
    c->rank = rank;
    c->nranks = nranks;
    *out = c;
    return SURFHIP_OK;
}

int surfhip_comm_destroy(surfhip_comm* c)
{
    if (!c) return SURFHIP_ERR_INVALID;
    const ncclResult_t r = ncclCommDestroy(c->nc);
    delete c;
    NCCLCHK(r);
    return SURFHIP_OK;
}

int surfhip_comm_rank(surfhip_comm* c, int* rank, int* nranks)
{
    if (!c) return SURFHIP_ERR_INVALID;
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    return SURFHIP_OK;
}

int surfhip_allgather(surfhip_comm* c, const void* send, size_t bytes, void* recv, void* stream)
{
    if (!c || !send || !recv || bytes == 0) return SURFHIP_ERR_INVALID;
    NCCLCHK(ncclAllGather(send, recv, bytes, ncclUint8, c->nc, (hipStream_t)stream));
    return SURFHIP_OK;
}

int surfhip_allreduce_sum_i64(surfhip_comm* c, long long* vals, int n, void* stream)
{
    if (!c || !vals || n < 1) return SURFHIP_ERR_INVALID;
    NCCLCHK(ncclAllReduce(vals, vals, (size_t)n, ncclInt64, ncclSum, c->nc, (hipStream_t)stream));
    return SURFHIP_OK;
}

int surfhip_comm_last_error(void) { return (int)g_last_nccl; }

}  // extern "C"
