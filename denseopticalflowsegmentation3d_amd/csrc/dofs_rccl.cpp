// dofs_rccl.cpp — libdofs_rccl.so: the C-ABI of include/dofs_rccl.h, the final gather of each frame's
// 3D-box records over RCCL (xGMI) for C / C++ hosts running one GPU per process. The box records of a
// batch are staged into one contiguous block per rank with dofs_batch_records_copy (stream-ordered, on
// the device), then one ncclGather (or ncclAllGather) moves the equal blocks; nothing is staged through
// the host. Blocks are a few hundred KB per rank at B = 96, so the collective is latency-bound: one
// call per batch, not one per frame.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <string>

#include "../../include/dofs_rccl.h"

struct dofs_comm {
    ncclComm_t c = nullptr;
    bool owned = false;
    int rank = 0, n = 1;
    void* buf = nullptr;  // this rank's staged block (grow-only)
    size_t cap = 0;
    std::string err;
};

namespace {
int fail(dofs_comm* c, int code, const std::string& msg) {
    if (c) c->err = msg;
    return code;
}
int nccl(dofs_comm* c, ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return DOFS_OK;
    return fail(c, DOFS_ERR_DEVICE, std::string(what) + ": " + ncclGetErrorString(r));
}
int fill(dofs_comm* c) {
    int rank = 0, n = 0;
    if (int rc = nccl(c, ncclCommUserRank(c->c, &rank), "ncclCommUserRank")) return rc;
    if (int rc = nccl(c, ncclCommCount(c->c, &n), "ncclCommCount")) return rc;
    c->rank = rank;
    c->n = n;
    return DOFS_OK;
}
}  // namespace

extern "C" {

int32_t dofs_comm_unique_id(uint8_t id[DOFS_COMM_ID_BYTES]) {
    static_assert(sizeof(ncclUniqueId) == DOFS_COMM_ID_BYTES, "ncclUniqueId size");
    if (!id) return DOFS_ERR_INVALID_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return DOFS_ERR_DEVICE;
    memcpy(id, &u, sizeof(u));
    return DOFS_OK;
}

int32_t dofs_comm_init(dofs_comm** comm, int32_t nranks, const uint8_t id[DOFS_COMM_ID_BYTES], int32_t rank,
                       int32_t device) {
    if (!comm || !id || nranks < 1 || rank < 0 || rank >= nranks) return DOFS_ERR_INVALID_ARG;
    *comm = nullptr;
    if (hipSetDevice(device) != hipSuccess) return DOFS_ERR_NO_DEVICE;
    dofs_comm* c = new dofs_comm;
    ncclUniqueId u;
    memcpy(&u, id, sizeof(u));
    if (nccl(c, ncclCommInitRank(&c->c, nranks, u, rank), "ncclCommInitRank") || fill(c)) {
        delete c;
        return DOFS_ERR_DEVICE;
    }
    c->owned = true;
    *comm = c;
    return DOFS_OK;
}

int32_t dofs_comm_init_local(dofs_comm** comms, int32_t n, const int32_t* devices) {
    if (!comms || n < 1 || !devices) return DOFS_ERR_INVALID_ARG;
    ncclComm_t* cs = new ncclComm_t[n];
    int* devs = new int[n];
    for (int i = 0; i < n; ++i) devs[i] = devices[i];
    const ncclResult_t r = ncclCommInitAll(cs, n, devs);
    delete[] devs;
    if (r != ncclSuccess) {
        delete[] cs;
        return DOFS_ERR_DEVICE;
    }
    for (int i = 0; i < n; ++i) {
        comms[i] = new dofs_comm;
        comms[i]->c = cs[i];
        comms[i]->owned = true;
        fill(comms[i]);
    }
    delete[] cs;
    return DOFS_OK;
}

int32_t dofs_comm_wrap(dofs_comm** comm, void* nccl_comm) {
    if (!comm || !nccl_comm) return DOFS_ERR_INVALID_ARG;
    dofs_comm* c = new dofs_comm;
    c->c = static_cast<ncclComm_t>(nccl_comm);
    c->owned = false;
    if (int rc = fill(c)) {
        delete c;
        return rc;
    }
    *comm = c;
    return DOFS_OK;
}

void dofs_comm_destroy(dofs_comm* comm) {
    if (!comm) return;
    if (comm->buf) (void)hipFree(comm->buf);
    if (comm->owned && comm->c) ncclCommDestroy(comm->c);
    delete comm;
}

int32_t dofs_comm_rank(const dofs_comm* comm, int32_t* rank, int32_t* nranks) {
    if (!comm) return DOFS_ERR_INVALID_ARG;
    if (rank) *rank = comm->rank;
    if (nranks) *nranks = comm->n;
    return DOFS_OK;
}

const char* dofs_comm_last_error(const dofs_comm* comm) { return comm ? comm->err.c_str() : "null communicator"; }

size_t dofs_records_block_bytes(int32_t frames, int32_t per_frame) {
    if (frames < 0 || per_frame < 0) return 0;
    return sizeof(int32_t) * (size_t)frames + sizeof(dofs_box_record) * (size_t)frames * (size_t)per_frame;
}

int32_t dofs_gather_bytes(dofs_comm* comm, const void* d_send, size_t bytes, int32_t root, void* d_recv,
                          void* stream) {
    if (!comm || !d_send || root >= comm->n) return fail(comm, DOFS_ERR_INVALID_ARG, "bad args");
    if ((root < 0 || root == comm->rank) && !d_recv) return fail(comm, DOFS_ERR_INVALID_ARG, "no receive buffer");
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (root >= 0)
        return nccl(comm, ncclGather(d_send, d_recv, bytes, ncclUint8, root, comm->c, s), "ncclGather");
    return nccl(comm, ncclAllGather(d_send, d_recv, bytes, ncclUint8, comm->c, s), "ncclAllGather");
}

int32_t dofs_gather_records(dofs_ctx* ctx, dofs_comm* comm, int32_t per_frame, int32_t root, void* d_recv,
                            void* stream) {
    if (!ctx || !comm || per_frame < 0) return fail(comm, DOFS_ERR_INVALID_ARG, "bad args");
    const int32_t B = dofs_batch_frames(ctx);
    if (B <= 0) return fail(comm, DOFS_ERR_INVALID_ARG, "no batch on the context");
    const size_t bytes = dofs_records_block_bytes(B, per_frame);
    if (bytes > comm->cap) {
        if (comm->buf) {
            (void)hipStreamSynchronize(static_cast<hipStream_t>(stream));  // an earlier gather may still read it
            (void)hipFree(comm->buf);
        }
        comm->buf = nullptr;
        comm->cap = 0;
        if (hipMalloc(&comm->buf, bytes) != hipSuccess) return fail(comm, DOFS_ERR_OOM, "hipMalloc");
        comm->cap = bytes;
    }
    const int rc = dofs_batch_records_copy(ctx, comm->buf, per_frame, stream);
    // DOFS_ERR_INVALID_RESULT: the batch's results are invalid and its block holds DOFS_RECORDS_INVALID counts.
    // The collective still runs (the other ranks are in it), so every receiver sees the invalid frames; the
    // error is returned after it. Other errors (DOFS_ERR_DEVICE: a HIP call failed) leave no block to send.
    if (rc && rc != DOFS_ERR_INVALID_RESULT)
        return fail(comm, rc, std::string("dofs_batch_records_copy: ") + dofs_last_error(ctx));
    const std::string copy_err = rc ? std::string("dofs_batch_records_copy: ") + dofs_last_error(ctx) : std::string();
    if (int g = dofs_gather_bytes(comm, comm->buf, bytes, root, d_recv, stream)) return g;
    return rc ? fail(comm, rc, copy_err) : DOFS_OK;
}

}  // extern "C"
