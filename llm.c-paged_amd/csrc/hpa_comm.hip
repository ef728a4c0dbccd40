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
#include <stdlib.h>
#include <string.h>

#include "hpa_internal.h"

namespace {
ncclComm_t g_comm = nullptr;
int g_nranks = 0, g_rank = -1;
// single-process form (hpa_comm_init_all): one communicator per device
ncclComm_t* g_all = nullptr;
int* g_all_dev = nullptr;
int g_all_n = 0;
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
    if (g_all) {  // the single-process set: every device's communicator
        ncclResult_t r = ncclSuccess;
        for (int i = 0; i < g_all_n; ++i)
            if (g_all[i]) {
                const ncclResult_t ri = ncclCommDestroy(g_all[i]);
                if (r == ncclSuccess) r = ri;
            }
        free(g_all);
        free(g_all_dev);
        g_all = nullptr;
        g_all_dev = nullptr;
        g_all_n = 0;
        g_comm = nullptr;
        g_nranks = 0;
        g_rank = -1;
        return r == ncclSuccess ? 0 : hpa_fail(__FILE__, __LINE__, ncclGetErrorString(r));
    }
    if (!g_comm) return 0;
    const ncclResult_t r = ncclCommDestroy(g_comm);
    g_comm = nullptr;
    g_nranks = 0;
    g_rank = -1;
    return r == ncclSuccess ? 0 : hpa_fail(__FILE__, __LINE__, ncclGetErrorString(r));
}

int hpa_comm_size(void) { return g_nranks; }
int hpa_comm_rank(void) { return g_rank; }

int hpa_comm_gather_layout(int nranks, int rank, int root, const size_t* bytes_per_rank, size_t* recv_off,
                           size_t* own_off) {
    if (nranks < 1 || rank < 0 || rank >= nranks || root < 0 || root >= nranks || !bytes_per_rank) return -1;
    size_t off = 0;
    int posts = 0;
    for (int r = 0; r < nranks; ++r) {
        if (recv_off) recv_off[r] = off;
        if (r == root && own_off) *own_off = off;
        if (r != root && bytes_per_rank[r]) ++posts;
        off += bytes_per_rank[r];
    }
    if (rank != root) return bytes_per_rank[rank] ? 1 : 0;
    return posts;
}

int hpa_comm_gather_plan(int nranks, int rank, int root, const size_t* bytes_per_rank, HpaCommOp* ops,
                         int max_ops) {
    if (nranks < 1 || rank < 0 || rank >= nranks || root < 0 || root >= nranks || !bytes_per_rank || max_ops < 0)
        return -1;
    int n = 0;
    const auto put = [&](int op, int peer, size_t off, size_t bytes) {
        if (ops && n < max_ops) ops[n] = HpaCommOp{op, peer, off, bytes};
        ++n;
    };
    if (rank != root) {
        if (bytes_per_rank[rank]) put(HPA_COMM_SEND, root, 0, bytes_per_rank[rank]);
    } else {
        size_t off = 0;  // rank order: rank q's rows at sum(bytes[0..q-1]) (hpa_comm_gather_layout)
        for (int q = 0; q < nranks; ++q) {
            if (q != root && bytes_per_rank[q]) put(HPA_COMM_RECV, q, off, bytes_per_rank[q]);
            off += bytes_per_rank[q];
        }
        size_t own = 0;
        for (int q = 0; q < root; ++q) own += bytes_per_rank[q];
        if (bytes_per_rank[root]) put(HPA_COMM_COPY, root, own, bytes_per_rank[root]);
    }
    return ops && n > max_ops ? -1 : n;
}

// Rank r sends its send_bytes to root, which places them at offset
// sum(bytes_per_rank[0..r-1]) of recv (rank order): the operations of
// hpa_comm_gather_plan, point-to-point ones inside one NCCL group, then the
// root's local copy.  Enqueued on `stream` (NULL = the library stream);
// asynchronous.
int hpa_comm_gatherv(const void* send, size_t send_bytes, void* recv, const size_t* bytes_per_rank, int root,
                     void* stream) {
    HPA_REQUIRE(g_comm, "comm_gatherv: hpa_comm_init first");
    HPA_REQUIRE(root >= 0 && root < g_nranks && bytes_per_rank, "comm_gatherv: bad root / counts");
    HPA_REQUIRE(bytes_per_rank[g_rank] == send_bytes, "comm_gatherv: send_bytes != bytes_per_rank[rank]");
    HPA_REQUIRE(g_rank != root || recv, "comm_gatherv: root needs a receive buffer");
    hipStream_t s = stream ? (hipStream_t)stream : hpa_stream();
    HpaCommOp* ops = (HpaCommOp*)malloc((size_t)g_nranks * sizeof(HpaCommOp));
    HPA_REQUIRE(ops, "comm_gatherv: out of host memory");
    const int n = hpa_comm_gather_plan(g_nranks, g_rank, root, bytes_per_rank, ops, g_nranks);
    ncclResult_t r = n < 0 ? ncclInvalidArgument : ncclGroupStart();
    const bool grouped = n >= 0 && r == ncclSuccess;
    for (int i = 0; i < n && r == ncclSuccess; ++i) {
        const HpaCommOp& o = ops[i];
        if (o.op == HPA_COMM_SEND) r = ncclSend(send, o.bytes, ncclChar, o.peer, g_comm, s);
        else if (o.op == HPA_COMM_RECV) r = ncclRecv((char*)recv + o.offset, o.bytes, ncclChar, o.peer, g_comm, s);
    }
    const ncclResult_t r2 = grouped ? ncclGroupEnd() : ncclSuccess;
    int copy_rc = 0;
    for (int i = 0; i < n && r == ncclSuccess && r2 == ncclSuccess; ++i)
        if (ops[i].op == HPA_COMM_COPY && (char*)recv + ops[i].offset != send)
            copy_rc |= hipMemcpyAsync((char*)recv + ops[i].offset, send, ops[i].bytes, hipMemcpyDeviceToDevice, s) !=
                       hipSuccess;
    free(ops);
    HPA_NCCL(r);
    HPA_NCCL(r2);
    HPA_REQUIRE(!copy_rc, "comm_gatherv: root's local copy failed");
    return 0;
}

// (a device word per call: rare calls -- timing --, and the current device
// may change between them in the single-process form)
int hpa_comm_allreduce_max(double* value) {
    HPA_REQUIRE(g_comm && value, "comm_allreduce_max: hpa_comm_init first");
    double* w = nullptr;
    HPA_CHECK(hipMalloc(&w, sizeof(double)));
    hipStream_t s = hpa_stream();
    int rc = hipMemcpyAsync(w, value, sizeof(double), hipMemcpyHostToDevice, s) != hipSuccess;
    const ncclResult_t r = rc ? ncclSuccess : ncclAllReduce(w, w, 1, ncclFloat64, ncclMax, g_comm, s);
    rc |= r != ncclSuccess;
    rc |= !rc && hipMemcpyAsync(value, w, sizeof(double), hipMemcpyDeviceToHost, s) != hipSuccess;
    rc |= hipStreamSynchronize(s) != hipSuccess;
    (void)hipFree(w);
    if (r != ncclSuccess) return hpa_fail(__FILE__, __LINE__, ncclGetErrorString(r));
    HPA_REQUIRE(!rc, "comm_allreduce_max: copy / sync failed");
    return 0;
}

int hpa_comm_barrier(void) {
    double v = 0.0;
    return hpa_comm_allreduce_max(&v);
}

int hpa_comm_init_all(int ndev, const int* devs) {
    HPA_REQUIRE(ndev >= 1 && devs, "comm_init_all: devices");
    HPA_REQUIRE(!g_comm && !g_all, "comm_init_all: a communicator exists (hpa_comm_destroy first)");
    g_all = (ncclComm_t*)calloc(ndev, sizeof(ncclComm_t));
    g_all_dev = (int*)malloc(ndev * sizeof(int));
    HPA_REQUIRE(g_all && g_all_dev, "comm_init_all: out of host memory");
    memcpy(g_all_dev, devs, ndev * sizeof(int));
    const ncclResult_t r = ncclCommInitAll(g_all, ndev, devs);
    if (r != ncclSuccess) {
        free(g_all);
        free(g_all_dev);
        g_all = nullptr;
        g_all_dev = nullptr;
        return hpa_fail(__FILE__, __LINE__, ncclGetErrorString(r));
    }
    g_all_n = ndev;
    return hpa_comm_use(0);
}

// an NCCL group around the calls between them (the single-process form: one
// thread posting every device's gather, which RCCL needs grouped or it
// blocks on the first device's send)
int hpa_comm_group_start(void) {
    HPA_NCCL(ncclGroupStart());
    return 0;
}

int hpa_comm_group_end(void) {
    HPA_NCCL(ncclGroupEnd());
    return 0;
}

int hpa_comm_use(int index) {
    HPA_REQUIRE(g_all && index >= 0 && index < g_all_n, "comm_use: hpa_comm_init_all first / index");
    if (hpa_get_device() != g_all_dev[index]) HPA_REQUIRE(hpa_init(g_all_dev[index]) == 0, "comm_use: device");
    g_comm = g_all[index];
    g_nranks = g_all_n;
    g_rank = index;
    return 0;
}

}  // extern "C"
