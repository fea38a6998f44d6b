// dofs_common.h — shared types of the MI355X clustering + lifting pipeline.
//
// The including translation unit defines, before including this header:
//   DOFS_HD                          function qualifier of per-element kernel bodies
//   DOFS_HDM                         host+device qualifier of pure math helpers (dofs_lift.h)
//   dofs_ld / dofs_st                relaxed agent-scope load / store of an int
//   dofs_ld64 / dofs_st64            relaxed agent-scope load / store of a 64-bit word
//   dofs_cas / dofs_exch             agent-scope compare-and-swap / exchange of an int
//   dofs_cas64                       agent-scope compare-and-swap of a 64-bit word
//   dofs_amin_u64 / dofs_amax_u64    agent-scope atomic min / max of a uint64
//   dofs_amin / dofs_amax / dofs_aadd / dofs_aor   agent-scope atomics on int
//   dofs_amin_u32                    agent-scope atomic min of a uint32
//   dofs_agg_size_bbox / dofs_agg_max / dofs_agg_min / dofs_agg_max_u64   keyed atomic updates
//                                    that a backend may aggregate across the lanes of a wave sharing
//                                    one key (called by every lane of the launch, `act` = participates)
// dofs_hip.hip maps them to HIP atomics on gfx950; the test-only host emulator maps them to plain
// sequential operations.
#pragma once

#include <stdint.h>

#include "../../include/dofs.h"

namespace dofs {

struct F2 {
    float x, y;
};

struct B4 {  // inclusive bbox with 16-bit coordinates (H, W < 32768)
    int16_t x0, y0, x1, y1;
};

struct I4 {
    int x0, y0, x1, y1;
};

// Value of one Kruskal-reconstruction-tree node = state of a union-find root right after the merge
// that created it (graph.cpp:170-218): size, union-by-rank root and rank, float running mean, bbox.
struct NodeVal {
    float mx, my;
    int size;
    int root;
    int16_t x0, y0, x1, y1;
    int rank;
    int pad;
};
static_assert(sizeof(NodeVal) == 32, "NodeVal must stay 32 bytes (one gather = 2 x dwordx4)");

// Replay output of the merge at one preorder position (Forest::merge's root state right after it):
// one 32-byte record instead of five arrays. 32 bytes, aligned: a record is one whole 32-byte sector and
// never shares one with another record. The replay hands records between waves with write-through
// stores and L2-served loads; a 24-byte form (round 5) failed intermittently (one illegal address and one
// wrong snapshot count in about fifty GPU runs, none in the 32-byte form) — likely a load of one record
// bringing a neighbour's not-yet-published bytes of a shared sector into the reader's L2.
struct alignas(16) RepVal {
    float mx, my;
    int rank, root;
    B4 bb;
    int pad0, pad1;
};
static_assert(sizeof(RepVal) == 32, "RepVal is one 32-byte record");

constexpr int kMaxTaps = 64;
constexpr int kRoundsMax = 40;        // Borůvka round flags per frame
constexpr int kCounters = 64;         // per-frame counter block (ints)
enum Counter {
    C_PATHS = 0,
    C_CAND = 1,
    C_SCORED = 2,
    C_QUAL = 3,
    C_SNAP = 4,
    C_MST = 5,
    C_SHORT = 6,
    C_LONG = 7,
    C_SQ = 8,     // C_SQ + (r + 1) % 3: short paths parked in replay round r (three rotating counters)
    C_PROG = 11,  // KRT sweep progress (blocks whose labels are published; k_krt_fused)
    C_FUSE = 12,  // frame 0 only: [C_FUSE] sweep claims, [C_FUSE + 1] LDS-KRT block claims
    C_TINY = 15,  // short heavy paths of at most kTinyPath merges (listed from the back of list_short)
    C_OVF = 14,   // snapshot count of a frame whose records overflowed the capacity (0: no overflow)
    C_ACT = 16,  // C_ACT + r: Borůvka round r found a cross-component edge (r < kRoundsMax)
    C_KEEP = 54,     // merges whose replay record the lean replay stores (size >= min_size; KPathInit)
    C_OVF_ANY = 56,  // frame 0 only: 1 if any frame of the batch overflowed its snapshot records
    C_LONGM = 57,    // merges on long heavy paths (replayed by the wave-per-path kernel)
    C_FLOWERR = 58,  // frame 0 only: the batch's results are invalid (bits kErrGiveUp, kErrRecord, kErrMst; dofs_kernels.h)
    C_ROOTL = 59,    // 1 + position in list_long of the frame's root heavy path (0: the root path is short)
    C_SORTFIX = 60,  // frame 0 only, 3 counters: pairs the MST sort fix-up moved, its fallback flag, barrier
    C_BMAX = 63      // the frame's largest |blurred flow component| (float bits, atomicMax by the HIP blur)
};
// Borůvka's round flags C_ACT + r use r < ceil(log2(H*W)) + 2 <= 28 (H*W < 2^26): C_KEEP sits above them
static_assert(C_ACT + 28 < C_KEEP, "counter layout");

constexpr uint32_t kNoEdge = 0xFFFFFFFFu;
constexpr int kIntMax = 0x7FFFFFFF;
// Pixels of a batch (B * H * W) at most: the dataflow replay's task words hold frame * H*W + path below
// kFlowLong = 2^30 and stay below its state words (kFlowDone = 2^31 - 16 and the open words above it) with
// the long bit set (static_assert in dofs_dataflow.h). 1080p: 517 frames (205 GB of input, which fits in HBM).
constexpr int64_t kMaxBatchPixels = ((int64_t)1 << 30) - 16;

// Linear dimensions of one frame and of the batch.
struct Dims {
    int H, W;
    int64_t N;   // pixels
    int64_t M;   // MST edges = merges = N - 1
    int64_t NL;  // KRT nodes = label space = N + M
    int64_t P2;  // power of two >= N (segment tree leaves)
    int B;       // frames in the batch
    int nbr8;
};

}  // namespace dofs
