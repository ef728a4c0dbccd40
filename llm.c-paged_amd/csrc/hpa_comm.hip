// hpa_comm.hip -- RCCL over xGMI for the sequence-sharded decode (SURVEY.md
// 8e).  One process per GPU; every rank decodes its own contiguous range of
// the batch on a private page pool with replicated weights, so a step has no
// exchange inside it.  The one collective is the north star's end-of-step
// gather of the logits (or of the greedy ids) to a root rank: a grouped
// ncclSend / ncclRecv gather (uneven row counts allowed), issued on a stream
// the caller names (the decode engine uses its communication stream so the
// gather of step k overlaps the kernels of step k+1).  Host code only; the
// reference has no collective outside the PyTorch trainer
// (train_gpt2.py:400-412).
#include <rccl/rccl.h>
#include <string.h>

#include "hpa_internal.h"

namespace {
ncclComm_t g_comm = nullptr;
int g_nranks = 0, g_rank = -1;
}  // namespace

#define HPA_NCCL(call)                                                                          \
    do {                                                                                        \
        ncclResult_t r_ = (call);                                                               \
        if (r_ != ncclSuccess) return hpa_fail(__FILE__, __LINE__, ncclGetErrorString(r_));     \
    } while (0)

extern "C" {

size_t hpa_comm_id_bytes(void) { return sizeof(ncclUniqueId); }

int hpa_comm_unique_id(void* id, size_t id_bytes) {
    HPA_REQUIRE(id && id_bytes >= sizeof(ncclUniqueId), "comm_unique_id: buffer of hpa_comm_id_bytes() bytes");
    ncclUniqueId u;
    HPA_NCCL(ncclGetUniqueId(&u));
    memcpy(id, &u, sizeof(u));
    return 0;
}

int hpa_comm_init(int nranks, int rank, const void* id) {
    HPA_REQUIRE(id && nranks >= 1 && rank >= 0 && rank < nranks, "comm_init: bad rank / size");
    HPA_REQUIRE(hpa_get_device() >= 0, "comm_init: hpa_init first (the communicator binds the current device)");
    HPA_REQUIRE(!g_comm, "comm_init: a communicator exists (hpa_comm_destroy first)");
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    HPA_NCCL(ncclCommInitRank(&g_comm, nranks, u, rank));
    g_nranks = nranks;
    g_rank = rank;
    return 0;
}

int hpa_comm_destroy(void) {
    if (!g_comm) return 0;
    const ncclResult_t r = ncclCommDestroy(g_comm);
    g_comm = nullptr;
    g_nranks = 0;
    g_rank = -1;
    return r == ncclSuccess ? 0 : hpa_fail(__FILE__, __LINE__, ncclGetErrorString(r));
}

int hpa_comm_size(void) { return g_nranks; }
int hpa_comm_rank(void) { return g_rank; }

// Rank r sends its send_bytes to root, which places them at offset
// sum(bytes_per_rank[0..r-1]) of recv (rank order).  Enqueued on `stream`
// (NULL = the library stream); asynchronous.
int hpa_comm_gatherv(const void* send, size_t send_bytes, void* recv, const size_t* bytes_per_rank, int root,
                     void* stream) {
    HPA_REQUIRE(g_comm, "comm_gatherv: hpa_comm_init first");
    HPA_REQUIRE(root >= 0 && root < g_nranks && bytes_per_rank, "comm_gatherv: bad root / counts");
    HPA_REQUIRE(bytes_per_rank[g_rank] == send_bytes, "comm_gatherv: send_bytes != bytes_per_rank[rank]");
    hipStream_t s = stream ? (hipStream_t)stream : hpa_stream();
    if (g_rank != root) {
        if (send_bytes) HPA_NCCL(ncclSend(send, send_bytes, ncclChar, root, g_comm, s));
        return 0;
    }
    HPA_REQUIRE(recv, "comm_gatherv: root needs a receive buffer");
    size_t off = 0;
    HPA_NCCL(ncclGroupStart());
    for (int r = 0; r < g_nranks; ++r) {
        if (r != root && bytes_per_rank[r])
            HPA_NCCL(ncclRecv((char*)recv + off, bytes_per_rank[r], ncclChar, r, g_comm, s));
        off += bytes_per_rank[r];
    }
    HPA_NCCL(ncclGroupEnd());
    off = 0;
    for (int r = 0; r < root; ++r) off += bytes_per_rank[r];
    if (send_bytes && (char*)recv + off != send)
        HPA_CHECK(hipMemcpyAsync((char*)recv + off, send, send_bytes, hipMemcpyDeviceToDevice, s));
    return 0;
}

}  // extern "C"
