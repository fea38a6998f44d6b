/*
 * dofs_rccl.h — C-ABI of the frame-parallel gather of 3D-box records over RCCL (xGMI), for C / C++ hosts
 * that drive one GPU per process through include/dofs.h (library: libdofs_rccl.so, which links librccl and
 * libdofs_hip.so; keeping it separate leaves libdofs_hip.so free of an RCCL dependency).
 *
 * Reference: the reference has no multi-GPU or collective code at all. Frames are
 * independent (main1's loop, cpp/src/segment.cpp:209-269, carries only the previous frame), so ranks shard
 * frames with no data-path collective and the only exchange is this final gather of each frame's 3D boxes
 * (north_star: "a final RCCL gather of 3D boxes over xGMI"). The Python host
 * (denseopticalflowsegmentation3d_amd/frames.py) does the same exchange through torch.distributed.
 *
 * Block layout (one per rank, the dofs_batch_records_copy layout): int32 counts[B] (snapshots per frame), then
 * B x per_frame dofs_box_record (the first per_frame records of each frame; unused records have slot -1).
 * Every rank must pass the same B (frames of its last batch) and per_frame: the collective moves equal blocks.
 */
#ifndef DOFS_RCCL_H
#define DOFS_RCCL_H

#include <stddef.h>
#include <stdint.h>

#include "dofs.h"

#ifdef __cplusplus
extern "C" {
#endif

#define DOFS_COMM_ID_BYTES 128 /* ncclUniqueId */

typedef struct dofs_comm dofs_comm;

/* ncclGetUniqueId: called by one rank, whose host then sends the bytes to the others by its own means. */
int32_t dofs_comm_unique_id(uint8_t id[DOFS_COMM_ID_BYTES]);
/* ncclCommInitRank on `device` (collective over the nranks processes). */
int32_t dofs_comm_init(dofs_comm** comm, int32_t nranks, const uint8_t id[DOFS_COMM_ID_BYTES], int32_t rank,
                       int32_t device);
/* A single-process communicator over n local devices (ncclCommInitAll); comms[i] gets device devices[i]. */
int32_t dofs_comm_init_local(dofs_comm** comms, int32_t n, const int32_t* devices);
/* Wrap a communicator the host created itself (an ncclComm_t); dofs_comm_destroy then leaves it alive. */
int32_t dofs_comm_wrap(dofs_comm** comm, void* nccl_comm);
void dofs_comm_destroy(dofs_comm* comm);
int32_t dofs_comm_rank(const dofs_comm* comm, int32_t* rank, int32_t* nranks);
const char* dofs_comm_last_error(const dofs_comm* comm);

/* Bytes of one rank's block for B frames and per_frame records each. */
size_t dofs_records_block_bytes(int32_t frames, int32_t per_frame);

/* The box records of ctx's last batch gathered over comm, stream-ordered on `stream` (hipStream_t or NULL):
 * root >= 0: ncclGather to rank `root`, d_recv (nranks blocks in rank order) is only written there and may be
 * NULL elsewhere; root < 0: ncclAllGather, every rank's d_recv receives all blocks. Returns what
 * dofs_batch_records_copy returns (DOFS_ERR_CAPACITY when a frame overflowed the snapshot capacity, before any
 * collective is issued — every rank sees its own overflow, so a host should agree on it before gathering;
 * DOFS_ERR_INVALID_RESULT after the collective, whose block from this rank then carries DOFS_RECORDS_INVALID
 * counts; any other copy error before it, with nothing sent), or DOFS_ERR_DEVICE if RCCL fails
 * (dofs_comm_last_error). */
int32_t dofs_gather_records(dofs_ctx* ctx, dofs_comm* comm, int32_t per_frame, int32_t root, void* d_recv,
                            void* stream);

/* Equal blocks of `bytes` from every rank (device buffers): gather to root (root >= 0) or all-gather. */
int32_t dofs_gather_bytes(dofs_comm* comm, const void* d_send, size_t bytes, int32_t root, void* d_recv,
                          void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DOFS_RCCL_H */
