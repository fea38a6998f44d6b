// dofs_dataflow.h — K5, the replay of Forest::merge (graph.cpp:170-218) along heavy paths, as ONE
// dataflow launch per batch (included by dofs_hip.hip; the test emulator keeps the round-based form,
// KReplay in dofs_kernels.h).
//
// Why: a heavy path advances until it meets a light child whose own path is not complete. The round
// launches park such a path until the next round, so a round lasts as long as the longest advance
// of any frame's path in it, and the batch pays the sum over rounds of those maxima (a kernel trace of
// the 96-frame 1080p bench: rounds 0, 7, 8 and 9 took 37.6, 13.8, 15.2 and 13.5 ms, 93 ms in all, while
// a frame's longest chain — its KRT height, ~370k merges — needs ~20 ms). Here a path that blocks
// registers itself on its light child and gives its wave away; the child's completion hands the
// parked path to whoever completed it, so every frame's chain runs as soon as its inputs exist and
// the batch takes about its longest chain.
//
// Tasks. A task is one heavy path of one frame, word t = f * N + j (path j of frame f, < 2^30) | kFlowLong
// for a long path (>= long_path merges, run by a whole wave as in k_replay_long1: 64 steps resolved in
// parallel per chunk, both mean chains in one instruction stream); short paths run one per lane.
//
// State word of a path top (state_at(): the top's record's first pad word): open (kIntMax / kPendLong from KPathInit) → the
// task word of the parent path parked on it (a light child has one parent position, so one waiter) →
// kFlowDone. The parker publishes its cursor and running state, then CASes its task word in; the
// completer publishes the top's record, then exchanges kFlowDone in and continues the waiter it got
// back (a lane a short waiter; a long waiter goes to the long-path queue, whose tickets the dedicated
// long workers hold). No task waits for another, so there is no deadlock and no residency requirement:
// short workers leave when the pool is empty and their lanes are done, long workers when every long
// path completed.
//
// Visibility inside the launch (MI355X_MICROARCH.md § visibility, cdna_hip_programming.md Guideline
// 16): every word handed between workgroups — records of path tops and parked states, cursors, state
// words, queue slots — is stored with agent-scope (sc1, write-through) stores, drained with
// s_waitcnt vmcnt(0) before the state word that signals it, and read only with agent-scope (sc1)
// loads, so no fence is needed. Everything else the launch reads was written by earlier launches.
#pragma once

namespace dofs {

constexpr int kFlowDone = 0x7FFFFFF0;  // state word of a completed path top (open words are above it)
constexpr int kFlowLong = 1 << 30;     // task word bit: a long path (run by a whole wave)
constexpr int kFlowIdMask = kFlowLong - 1;
// every task word (< kMaxBatchPixels, | kFlowLong for a long path) is below every state word (api_run refuses
// larger batches)
static_assert(kMaxBatchPixels <= (long long)kFlowDone - kFlowLong, "task words must stay below kFlowDone");

// control block (ints), zeroed and filled by k_flow_prep each launch; per-frame prefix sums follow. Every
// word that waves update or poll sits on a 256-byte line of its own: thousands of waves touch them, and
// words sharing a line share its memory channel's queue (a CAS storm on the queue head there stalled
// the pool claims next to it).
constexpr int kFlowLine = 64;  // ints per line
enum FlowCtlIdx {
    FC_LONG_NEXT = 0 * kFlowLine,   // initial long pool: next unclaimed index
    FC_SHORT_NEXT = 1 * kFlowLine,  // initial short pool (tiny paths of every frame first, then the others)
    FC_QHEAD = 2 * kFlowLine,       // long-path queue (slots in w.bw, dead after the MST): head / tail
    FC_QTAIL = 3 * kFlowLine,
    FC_ERR = 4 * kFlowLine,         // a bounded wait gave up (results invalid; reported through C_FLOWERR)
    FC_LDONE = 5 * kFlowLine,       // long paths completed
    FC_NL = 7 * kFlowLine,          // read-only after k_flow_prep: pool sizes (long, tiny, other short)
    FC_NT = FC_NL + 1,
    FC_NS = FC_NL + 2,
    FC_QCAP = FC_NL + 3,            // queue slots: B * N (w.bw); tickets and pushes stay below it
    FC_NLPOOL = FC_NL + 4,          // initial long pool: B root-path entries, then the frames' other long paths
    FC_FS = 8 * kFlowLine,          // the launch anatomy: FS_N u64 counters, one 256-byte line each (FlowStat)
    FC_HDR = FC_FS + 28 * 64,       // then pl[B + 1], pt[B + 1], ps[B + 1]
};
inline int g_flow_order = 0;  // host: the two launches' order (dofs_debug_flow_order; 0 = side by side)
// host: constant-key chunks in the long-path loop (flow_long; 1 = on, the default: 96 % of the chunks, one 4K
// frame's replay 93 → 72 ms). dofs_debug_replay_keyfast(0) runs every chunk with the key update, the test of
// tests/test_gpu_replay_modes.py that the two give identical merge events.
inline int g_keyfast = 1;

// launch anatomy (a few atomics per task, not per step): per launch, in the context's control block
// (FC_FS; so two contexts on one device never mix their counts), read by dofs_debug_flow_stats
// (tools/flow_stats.py) after the launch
constexpr int kFsStride = 32;  // u64 per stat: one 256-byte line each
enum FlowStat {
    FS_T0 = 0,         // first wave start (100 MHz wall clock, min)
    FS_T_SHORT = 1,    // last short worker done (max)
    FS_T_LONG = 2,     // last long-path completion (max)
    FS_T_EXIT = 3,     // last wave exit (max)
    FS_LRUNS = 4,      // flow_long calls
    FS_LPARKS = 5,     // long paths parked
    FS_LCHUNKS = 6,    // 64-step chunks of long paths
    FS_PUSH = 7,       // long waiters queued by lanes
    FS_INJECT = 8,     // short waiters handed to a short round by a long completion
    FS_LDONE = 9,      // long completions
    FS_LTICKS = 10,    // wall time inside flow_long, summed over waves
    FS_SROUNDS = 11,   // flow_short calls
    FS_STICKS = 12,    // wall time inside flow_short, summed over waves
    FS_LSTEPS = 13,    // merges replayed by long paths
    FS_T_ROOT = 14,    // last completion of a frame's root heavy path (top at preorder 0; max)
    FS_RPARKS = 15,    // parks of root heavy paths
    FS_RSTEPS = 16,    // merges replayed by root heavy paths
    FS_RCHUNKS = 17,   // 64-step chunks of root heavy paths
    // measurement build only (-DDOFS_FLOW_PROF, `make prof`): 100 MHz ticks of the long-path chunk loop,
    // summed over waves — the steps alone, the tail (bbox scan, record stores, the hand-over of a
    // finished or blocked chunk), and the next chunk's resolve (its global loads and the waits on them)
    FS_P_STEPS = 18,
    FS_P_TAIL = 19,
    FS_P_NEXT = 20,
    FS_KFAST = 21,     // long-path chunks run with a constant key (no step reaches the carried rank)
    FS_RESTARTS = 22,  // pipelined resolve: stage fills (a run's first chunk, a re-resolve after a park)
    // measurement build, wave pairs (flow_pair): C's and H's ticks waiting at the chunk barriers
    FS_P_CWAIT = 23,
    FS_P_HWAIT = 24,
    FS_N = 28
};
static_assert(FS_N * kFsStride * 2 == FC_HDR - FC_FS, "FlowStat block size");
__device__ inline unsigned long long* fs_at(int* ctl, int i) {
    return reinterpret_cast<unsigned long long*>(ctl + FC_FS) + i * kFsStride;
}
__device__ inline unsigned long long fs_now() { return __builtin_amdgcn_s_memrealtime(); }
__device__ inline void fs_add(int* ctl, int i, unsigned long long v) { atomicAdd(fs_at(ctl, i), v); }
__device__ inline void fs_min(int* ctl, int i, unsigned long long v) { atomicMin(fs_at(ctl, i), v); }
__device__ inline void fs_max(int* ctl, int i, unsigned long long v) { atomicMax(fs_at(ctl, i), v); }

__device__ inline int f_ld(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline void f_st(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline unsigned long long f_ld64(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void f_st64(unsigned long long* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline void f_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// a poll of a word other workgroups update with atomics, read by an atomic (or 0): the value at the
// coherence point, whatever copy of the line this XCD's L2 holds (the idle long workers' polls of the
// queue and completion counters and of queue slots; a few per microsecond at most, so the cost is nil)
__device__ inline int f_poll(int* p) {
    return __hip_atomic_fetch_or(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ inline unsigned long long f_poll64(unsigned long long* p) {
    return __hip_atomic_fetch_or(p, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a 16-byte write-through (sc1) store: one global_store_dwordx4 (HIP has no 16-byte atomic store). It
// returns nothing, so the compiler needs no wait for it; f_drain's explicit vmcnt(0) covers it like any store
__device__ inline void f_st128(void* p, unsigned a, unsigned b, unsigned c, unsigned e) {
    typedef unsigned u4 __attribute__((ext_vector_type(4)));
    const u4 v = {a, b, c, e};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
// a RepVal handed to another workgroup: its 24 bytes as one 16-byte and one 8-byte write-through store (two
// sector writes; three 8-byte stores were three), never touching the pads — the first is a path top's state
// word (state_at), which a parker may be CASing meanwhile. Read back by three 8-byte loads (rv_fetch).
__device__ inline void rv_publish(RepVal* p, float mx, float my, int rank, int root, B4 bb) {
    f_st128(p, __float_as_uint(mx), __float_as_uint(my), (unsigned)rank, (unsigned)root);
    unsigned long long b;
    __builtin_memcpy(&b, &bb, 8);
    f_st64(reinterpret_cast<unsigned long long*>(p) + 2, b);
}
__device__ inline RepVal rv_fetch(const RepVal* p) {
    const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long a = f_ld64(q), b = f_ld64(q + 1), c = f_ld64(q + 2);
    RepVal r;
    r.mx = __uint_as_float((unsigned)a);
    r.my = __uint_as_float((unsigned)(a >> 32));
    r.rank = (int)(unsigned)b;
    r.root = (int)(unsigned)(b >> 32);
    __builtin_memcpy(&r.bb, &c, 8);
    r.pad0 = r.pad1 = 0;
    return r;
}

// the state below a cursor q: the bottom leaf's singleton set (static), or a record a parker published
__device__ inline void flow_start(const Ws& w, int f, int64_t qb, float* mx, float* my, int* rank, int* root, B4* bb) {
    const Dims& d = w.d;
    const int64_t lb = f * d.NL;
    const int x = w.ord[lb + qb];
    if (x < d.N) {
        path_start(w, f, qb, mx, my, rank, root, bb);
        return;
    }
    const RepVal v = rv_fetch(w.Rv + lb + qb);
    *mx = v.mx;
    *my = v.my;
    *rank = v.rank;
    *root = v.root;
    *bb = v.bb;
}

__device__ inline int flow_frame(const int* pre, int B, int i) {  // largest f with pre[f] <= i
    int lo = 0, hi = B;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pre[mid] <= i)
            lo = mid;
        else
            hi = mid;
    }
    return lo;
}
// Initial long pool entry i: entries [0, B) are the frames' root heavy paths (the KRT root's chain, the
// longest of a frame: started first), the rest every frame's other long paths (pl: their prefix sums).
// -1: frame i has no long path.
__device__ inline int flow_long_task(const Ws& w, const int* ctl, int i) {
    const int B = w.d.B;
    const int* pl = ctl + FC_HDR;
    int f, k;
    if (i < B) {
        f = i;
        k = -1;
        if (w.C(f)[C_LONG] == 0) return -1;
    } else {
        f = flow_frame(pl, B, i - B);
        k = i - B - pl[f];  // among the frame's long paths other than its first
    }
    const int rp = w.C(f)[C_ROOTL] > 0 ? w.C(f)[C_ROOTL] - 1 : 0;  // the entry taken first
    const int idx = k < 0 ? rp : (k < rp ? k : k + 1);
    const int j = w.list_long[f * w.d.N + idx];
    return (int)(f * w.d.N + j) | kFlowLong;
}
__device__ inline int flow_short_task(const Ws& w, const int* ctl, int i) {
    const int B = w.d.B;
    const int nt = ctl[FC_NT];
    if (i < nt) {
        const int* pt = ctl + FC_HDR + (B + 1);
        const int f = flow_frame(pt, B, i);
        const int j = w.list_short[f * w.d.N + w.d.N - 1 - (i - pt[f])];
        return (int)(f * w.d.N + j);
    }
    const int* ps = ctl + FC_HDR + 2 * (B + 1);
    const int f = flow_frame(ps, B, i - nt);
    const int j = w.list_short[f * w.d.N + (i - nt - ps[f])];
    return (int)(f * w.d.N + j);
}

// one thread: zero the control words, prefix sums of the per-frame pool sizes
__global__ void k_flow_prep(Ws w, int* ctl) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const int B = w.d.B;
    int* pl = ctl + FC_HDR;
    int* pt = pl + (B + 1);
    int* ps = pt + (B + 1);
    int sl = 0, st = 0, ss = 0;
    for (int f = 0; f < B; ++f) {
        pl[f] = sl;
        pt[f] = st;
        ps[f] = ss;
        sl += w.C(f)[C_LONG] > 0 ? w.C(f)[C_LONG] - 1 : 0;
        st += w.C(f)[C_TINY];
        ss += w.C(f)[C_SHORT];
    }
    pl[B] = sl;
    pt[B] = st;
    ps[B] = ss;
    for (int k = 0; k < FC_HDR; ++k) ctl[k] = 0;
    *fs_at(ctl, FS_T0) = ~0ull;
    int nl = 0;
    for (int f = 0; f < B; ++f) nl += w.C(f)[C_LONG];
    ctl[FC_NL] = nl;
    ctl[FC_NLPOOL] = B + sl;
    ctl[FC_NT] = st;
    ctl[FC_NS] = ss;
    ctl[FC_QCAP] = (int)(B * w.d.N);
}

// The waiter a completion's exchange returned from its top's state word: -1 if none was parked there (open
// words are above kFlowDone), else a task word of this batch — a word outside it (never seen) is a give-up, not
// a task to index by
__device__ inline int flow_waiter(const Ws& w, int* ctl, int old) {
    if (old >= kFlowDone) return -1;
    if (old < 0 || (long long)(old & kFlowIdMask) >= (long long)w.d.B * w.d.N) {
        f_st(ctl + FC_ERR, 1);
        return -1;
    }
    return old;
}

__device__ inline void flow_push(const Ws& w, int* ctl, unsigned epoch, int t) {
    const int s = atomicAdd(ctl + FC_QTAIL, 1);
    if (s >= ctl[FC_QCAP]) {  // (never: a push resumes a path parked on a completed top, < B * N of them)
        f_st(ctl + FC_ERR, 1);
        return;
    }
    f_st64(w.bw + s, ((unsigned long long)epoch << 32) | (unsigned)t);
}
// Resolve position p of a long path (one lane per step, as one_resolve); light children through the
// state words and published records.
__device__ inline int flow_resolve(const Ws& w, int64_t lb, int p, int top, OneRec* o, B4* lbb, int accept = -1) {
    lbb->x0 = lbb->y0 = 0x7fff;
    lbb->x1 = lbb->y1 = -1;
    if (p < top) return 0;
    const StepV in = step_v(w.In[lb + p], p, w.d.W);
    int meta = in.meta;
    int lrank = 0, lroot = in.lb;
    if (in.meta & kStepDyn) {
        const int lq = in.lb;
        if (p != accept && f_ld(state_at(w, lb + lq)) != kFlowDone) return meta;  // accept: seen done by a CAS
        const RepVal lv = rv_fetch(w.Rv + lb + lq);
        o->h[0].wb = lv.mx * (float)in.la;
        o->h[1].wb = lv.my * (float)in.la;
        lrank = lv.rank;
        lroot = lv.root;
        *lbb = lv.bb;
    } else {
        o->h[0].wb = in.wbx;
        o->h[1].wb = in.wby;
        lbb->x0 = lbb->x1 = (int16_t)(in.la & 0xffff);
        lbb->y0 = lbb->y1 = (int16_t)(in.la >> 16);
    }
    meta |= kLongOk;
    o->h[0].fs = o->h[1].fs = in.fs;
    o->h[0].r = o->h[1].r = in.r;
    o->pad = 0;
    o->lk = rk_pack(lrank, lroot);
    o->lkp = o->lk + (1u << kRankShift);
    o->bm = (meta & kStepB) ? ~0u : 0u;
    return meta;
}

// The pipelined resolve of a long path's chunks (flow_long). Resolving a chunk is three dependent
// global round trips — its StepIn records, then the state words of its dynamic light children, then the
// records of those that are done (rv_fetch only after the state word was seen done: the publisher wrote
// the record before the state word) — and the synchronous form paid all three at the top of every
// chunk, before its 64 steps (about three times the steps' own time). Here chunk q - 64 d of the lane's
// path runs stage 4 - d while chunk q is stepped: d = 3 loads the StepIn records, d = 2 the state words,
// d = 1 the records, and chunk q - 64 is built into LDS from them at the next chunk's start. Each stage's
// loads have one chunk's steps to arrive; a restart (a task's first chunk, or a re-resolve after a park
// that found its child done) fills the stages synchronously.
// Branch-free loads: a lane that needs none still loads (no loaded register is merged with a constant at a
// branch join — the merge made the compiler wait for the load right after issuing it). Its StepIn load reads
// its path top's record, a line the wave reads anyway; its state-word and record loads read g_flow_none, a
// line that is never written, so no wave ever loads a handed-off sector (a path top's state word and record)
// before it is published — only the lanes whose light child it is load it, the record after its state word
// read done (round 5 pointed these don't-care loads at the path's own unpublished top).
__device__ RepVal g_flow_none;  // zero, never written
__device__ inline StepIn pipe_in(const Ws& w, int64_t lb, int p, int top) {
    return w.In[lb + (p >= top ? p : top)];  // (p < top: meta is ignored, pipe_build checks p)
}
__device__ inline int pipe_rdy(const Ws& w, int64_t lb, const StepIn& in, int p, int top) {
    const bool dyn = p >= top && (step_meta(in) & kStepDyn);
    return f_ld(dyn ? state_at(w, lb + step_lq(in, p)) : &g_flow_none.pad0);
}
__device__ inline RepVal pipe_rv(const Ws& w, int64_t lb, const StepIn& in, int rdy, int p, int top) {
    const bool need = p >= top && (step_meta(in) & kStepDyn) && rdy == kFlowDone;
    return rv_fetch(need ? w.Rv + lb + step_lq(in, p) : &g_flow_none);
}
// flow_resolve from the pipeline's loaded values (same record, same meta)
__device__ inline int pipe_build(const Ws& w, const StepIn& sin, int rdy, const RepVal& lv, int p, int top, OneRec* o,
                                 B4* lbb) {
    lbb->x0 = lbb->y0 = 0x7fff;
    lbb->x1 = lbb->y1 = -1;
    if (p < top) return 0;
    const StepV in = step_v(sin, p, w.d.W);
    int meta = in.meta;
    int lrank = 0, lroot = in.lb;
    if (in.meta & kStepDyn) {
        // blocked (the chunk ends here; the park re-checks the state). The record is used only where the
        // state word it was loaded after read done (pipe_rv); elsewhere the load read another line.
        if (rdy != kFlowDone) return meta;
        o->h[0].wb = lv.mx * (float)in.la;
        o->h[1].wb = lv.my * (float)in.la;
        lrank = lv.rank;
        lroot = lv.root;
        *lbb = lv.bb;
    } else {
        o->h[0].wb = in.wbx;
        o->h[1].wb = in.wby;
        lbb->x0 = lbb->x1 = (int16_t)(in.la & 0xffff);
        lbb->y0 = lbb->y1 = (int16_t)(in.la >> 16);
    }
    meta |= kLongOk;
    o->h[0].fs = o->h[1].fs = in.fs;
    o->h[0].r = o->h[1].r = in.r;
    o->pad = 0;
    o->lk = rk_pack(lrank, lroot);
    o->lkp = o->lk + (1u << kRankShift);
    o->bm = (meta & kStepB) ? ~0u : 0u;
    return meta;
}

// The chain of one 64-step chunk (Forest::merge's running mean and union-by-rank key, graph.cpp:177-213):
// n steps of the records c[0..n), lane parity h carrying the x (h = 0) or y mean in v, and the key K.
// fastc (a constant-key chunk: no step's light key reaches K's rank): the mean chain alone — one LDS read,
// five VALU and a quarter LDS store per step instead of ~16 instructions with the key update — and its
// values as two rows of 64 floats in ob's storage (x row, y row); else {v, K} per step in ob[2 k + h].
__device__ __forceinline__ void chain_chunk(const OneRec* c, OneOut* ob, int n, bool fastc, int h, float& v,
                                            unsigned& K) {
    auto step = [&](int k, uint4 a, OneHalf b) {  // a = {lk, bm, lkp}, b = {r, wb, fs}
        v = (float)((double)(v * b.fs + b.wb) * b.r);
        const unsigned lk = a.x, bm = a.y, lkp = a.z;
        unsigned eq = (bm & lkp) | (~bm & (K + (1u << kRankShift)));
        unsigned ne = K > lk ? K : lk;
        asm volatile("" : "+v"(eq), "+v"(ne));
        K = (K ^ lk) < (1u << kRankShift) ? eq : ne;
        OneOut o;
        o.v = v;
        o.k = K;
        ob[2 * k + h] = o;
    };
    auto lda = [&](int k) { return *reinterpret_cast<const uint4*>(&c[k]); };
    if (fastc) {
        // The mean chain alone: per step one ds_read_b128 of the lane's half record, the five chain
        // ops, and the value (no key: it is K for the whole chunk) into the chunk's output slot. The
        // records run through three 4-step register sets: a set is reloaded 4 to 8 steps ahead of
        // its use (~90-170 cycles against the ~50-cycle LDS latency), and the sched barriers keep
        // the compiler from sinking those loads next to their uses (round 3's ISA had them issued
        // one to three steps ahead: the LDS latency was exposed twice per 8 steps).
        // values only, as two rows of 64 floats in ob's storage (x row, y row): four steps' values
        // are contiguous, one ds_write_b128 per 4 steps
        float* fvh = reinterpret_cast<float*>(ob) + 64 * h;
        const OneHalf* ch = &c[0].h[h];
        auto ld = [&](int k) { return *reinterpret_cast<const OneHalf*>(reinterpret_cast<const char*>(ch) + k * (int)sizeof(OneRec)); };
        auto chain = [&](const OneHalf& b) {
            v = (float)((double)(v * b.fs + b.wb) * b.r);
            return v;
        };
        auto stepf = [&](int k, const OneHalf& b) { fvh[k] = chain(b); };
        auto step4 = [&](int k, const OneHalf& a0, const OneHalf& a1, const OneHalf& a2, const OneHalf& a3) {
            float4 o;
            o.x = chain(a0);
            o.y = chain(a1);
            o.z = chain(a2);
            o.w = chain(a3);
            *reinterpret_cast<float4*>(fvh + k) = o;
        };
        // 8 steps per iteration in two 4-step register sets, each loaded 4 steps (~90 cycles) ahead of
        // its use; the sched barriers pin the loads there (round 3's ISA had the compiler sink them to
        // one to three steps ahead of their use: the LDS latency was exposed twice per 8 steps). The
        // sets are not rotated across iterations (a rotating ring compiled to v_mov_b64 copies, and a
        // fully unrolled chunk to AGPR spills)
        OneHalf b0 = ld(0), b1 = ld(1), b2 = ld(2), b3 = ld(3);
        int k = 0;
        for (; k + 8 <= n; k += 8) {
            const OneHalf d0 = ld(k + 4), d1 = ld(k + 5), d2 = ld(k + 6), d3 = ld(k + 7);
            __builtin_amdgcn_sched_barrier(0);
            step4(k, b0, b1, b2, b3);
            __builtin_amdgcn_sched_barrier(0);
            b0 = ld(k + 8), b1 = ld(k + 9), b2 = ld(k + 10), b3 = ld(k + 11);
            __builtin_amdgcn_sched_barrier(0);
            step4(k + 4, d0, d1, d2, d3);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (k + 4 <= n) {
            const OneHalf d0 = ld(k + 4), d1 = ld(k + 5), d2 = ld(k + 6);
            step4(k, b0, b1, b2, b3);
            if (k + 4 < n) stepf(k + 4, d0);
            if (k + 5 < n) stepf(k + 5, d1);
            if (k + 6 < n) stepf(k + 6, d2);
        } else {
            if (k < n) stepf(k, b0);
            if (k + 1 < n) stepf(k + 1, b1);
            if (k + 2 < n) stepf(k + 2, b2);
        }
    } else {
    // two register sets, each reloaded right after its last use (4 steps ahead of its next use): no
    // loop-carried copies (the single-set form with next-group temporaries compiled to ~4 v_mov per step)
    int k = 0;
    uint4 a0 = lda(0), a1 = lda(1), a2 = lda(2), a3 = lda(3);
    OneHalf b0 = c[0].h[h], b1 = c[1].h[h], b2 = c[2].h[h], b3 = c[3].h[h];
    for (; k + 8 <= n; k += 8) {
        const int m = k + 4, m2 = (k + 8) & 63;
        const uint4 e0 = lda(m), e1 = lda(m + 1), e2 = lda(m + 2), e3 = lda(m + 3);
        const OneHalf d0 = c[m].h[h], d1 = c[m + 1].h[h], d2 = c[m + 2].h[h], d3 = c[m + 3].h[h];
        step(k, a0, b0);
        step(k + 1, a1, b1);
        step(k + 2, a2, b2);
        step(k + 3, a3, b3);
        a0 = lda(m2), a1 = lda(m2 + 1), a2 = lda(m2 + 2), a3 = lda(m2 + 3);
        b0 = c[m2].h[h], b1 = c[m2 + 1].h[h], b2 = c[m2 + 2].h[h], b3 = c[m2 + 3].h[h];
        step(k + 4, e0, d0);
        step(k + 5, e1, d1);
        step(k + 6, e2, d2);
        step(k + 7, e3, d3);
    }
    if (k + 4 <= n) {
        step(k, a0, b0);
        step(k + 1, a1, b1);
        step(k + 2, a2, b2);
        step(k + 3, a3, b3);
        k += 4;
    }
    for (; k < n; ++k) step(k, lda(k), c[k].h[h]);
    }
}

// A long path (task word t) on this wave, from its cursor: returns the task word of the parent path
// that was parked on its top (to run next), or -1 (parked itself, or completed with nobody waiting).
__device__ int flow_long(const Ws& w, int* ctl, int t, OneRec (*buf)[64], OneOut* ob, int keyfast) {
    const Dims& d = w.d;
    const int g = t & kFlowIdMask;
    const int f = g / (int)d.N, j = g - f * (int)d.N;
    int* curp = w.cur + f * d.N + j;
    const int lane = threadIdx.x & 63;
    int q = f_ld(curp);
    const int top = w.ptop[f * d.N + j];
    if (q < top) return -1;  // (never: a task is handed out only while its path is not complete)
    const int64_t lb = f * d.NL;
    const int h = lane & 1;
    float v;
    unsigned K;
    B4 bb;
    {
        float mx, my;
        int rank, root;
        flow_start(w, f, q + 1, &mx, &my, &rank, &root, &bb);
        v = h ? my : mx;
        K = rk_pack(rank, root);
    }
    int cb = 0;
    OneRec rec;
    B4 lbb;
    int meta = flow_resolve(w, lb, q - lane, top, &rec, &lbb);
    buf[cb][lane] = rec;
    unsigned curlk = rec.lk;  // this lane's step key in the current chunk (valid for lanes < n)
    unsigned chunks = 0, steps = 0, kfast = 0, restarts = 1;  // anatomy, added once per call
#ifdef DOFS_FLOW_PROF
    unsigned long long p_steps = 0, p_tail = 0, p_next = 0, p_t = wall_clock64();
#define FLOW_PROF_MARK(acc)                                 \
    do {                                                    \
        const unsigned long long p_now = wall_clock64();   \
        acc += p_now - p_t;                                 \
        p_t = p_now;                                        \
    } while (0)
#else
#define FLOW_PROF_MARK(acc) \
    do {                    \
    } while (0)
#endif
    auto tally = [&]() {
        if (lane == 0) {
#ifdef DOFS_FLOW_PROF
            fs_add(ctl, FS_P_STEPS, p_steps);
            fs_add(ctl, FS_P_TAIL, p_tail);
            fs_add(ctl, FS_P_NEXT, p_next);
#endif
            fs_add(ctl, FS_LCHUNKS, chunks);
            fs_add(ctl, FS_LSTEPS, steps);
            fs_add(ctl, FS_KFAST, kfast);
            fs_add(ctl, FS_RESTARTS, restarts);
            if (top == 0) {
                fs_add(ctl, FS_RCHUNKS, chunks);
                fs_add(ctl, FS_RSTEPS, steps);
            }
        }
    };
    // the resolve stages in named registers rotated by a three-way unroll (as flow_pair's: a register copy of
    // an in-flight load waits for it, so the rotating form exposed a memory round trip per chunk): in1 / in2 /
    // in3 the StepIn records of chunks q - 64 / - 128 / - 192, rdy1 / rdy2 the state words, rv the light
    // records of chunk q - 64
    StepIn i0, i1, i2;
    int r0, r1, r2;
    RepVal rv;
    auto restart_stages = [&](int qq) {
        i0 = pipe_in(w, lb, qq - 64 - lane, top);
        i1 = pipe_in(w, lb, qq - 128 - lane, top);
        i2 = pipe_in(w, lb, qq - 192 - lane, top);
        r0 = pipe_rdy(w, lb, i0, qq - 64 - lane, top);
        r1 = pipe_rdy(w, lb, i1, qq - 128 - lane, top);
        rv = pipe_rv(w, lb, i0, r0, qq - 64 - lane, top);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing in flight where this path meets the back edge
    };
    restart_stages(q);
    int ret = -1;
    // one chunk: 0 = continue, 1 = the task ended (ret), 2 = re-resolved after a park found its child done
    auto iter = [&](StepIn& in1, StepIn& in2, StepIn& in3, int& rdy1, int& rdy2, int& rdy3) -> int {
        OneRec nrec;
        B4 nlbb;
        const int nmeta = pipe_build(w, in1, rdy1, rv, q - 64 - lane, top, &nrec, &nlbb);
        rv = pipe_rv(w, lb, in2, rdy2, q - 128 - lane, top);  // issued now, used a chunk later
        rdy3 = pipe_rdy(w, lb, in3, q - 192 - lane, top);
        in1 = pipe_in(w, lb, q - 256 - lane, top);  // (in1 was consumed by pipe_build)
        const unsigned long long blocked = __ballot(!(meta & kLongOk));
        const unsigned long long tops = __ballot((meta & kLongOk) && (meta & kStepTop));
        const int fb = blocked ? __ffsll((long long)blocked) - 1 : 64;
        const int ft = tops ? __ffsll((long long)tops) - 1 : 64;
        const int finished = ft < fb;
        const int n = finished ? ft + 1 : fb;
        ++chunks;
        steps += n;
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this chunk's LDS records have landed
        __builtin_amdgcn_wave_barrier();
        FLOW_PROF_MARK(p_next);  // the next chunk's resolve (its global loads and their waits)
        const OneRec* c = buf[cb];
        // Constant-key chunks: union by rank (graph.cpp:177-182, 210-213) leaves the carried key K
        // unchanged at a step whose light child has a lower rank (max(K, lk) = K). A lane checks its
        // own step against K's rank; when no step of the chunk reaches it (the common case: after
        // a path's first steps its light children are mostly pixels, rank 0), every step's key is K and
        // the loop carries only the mean chain (chain_chunk)
        const unsigned krank = K & ~((1u << kRankShift) - 1);
        const bool fastc = keyfast && __ballot(lane < n && curlk >= krank) == 0;
        if (fastc) ++kfast;
        chain_chunk(c, ob, n, fastc, h, v, K);
        FLOW_PROF_MARK(p_steps);
        B4 obb;
        {  // bbox: inclusive prefix join over the chunk (lane = step), then the carried box
            B4 x = lbb;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const B4 y = bb_shfl_up(x, o);
                if (lane >= o) x = bb_join(x, y);
            }
            x = bb_join(x, bb);
            obb = x;
            const int src = n > 0 ? n - 1 : 0;
            const int lo = __shfl((int)((unsigned short)x.x0 | ((unsigned)(unsigned short)x.y0 << 16)), src, 64);
            const int hi = __shfl((int)((unsigned short)x.x1 | ((unsigned)(unsigned short)x.y1 << 16)), src, 64);
            if (n > 0) {
                bb.x0 = (int16_t)(lo & 0xffff);
                bb.y0 = (int16_t)(lo >> 16);
                bb.x1 = (int16_t)(hi & 0xffff);
                bb.y1 = (int16_t)(hi >> 16);
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // the chunk's output records are in LDS
        __builtin_amdgcn_wave_barrier();
        if (lane < n) {
            // a constant-key chunk stored only the values (two rows), its key is the carried one
            const float* fv = reinterpret_cast<const float*>(ob);
            const OneOut sx = ob[2 * lane], sy = ob[2 * lane + 1];
            const float vx = fastc ? fv[lane] : sx.v, vy = fastc ? fv[64 + lane] : sy.v;
            const unsigned kk = fastc ? K : sx.k;
            const int rank = (int)(kk >> kRankShift), root = (int)(kk & ((1u << kRankShift) - 1));
            RepVal* dst = w.Rv + lb + q - lane;
            if (lane == n - 1 && (finished || n < 64)) {  // the top's record (parent path) or a parked state
                rv_publish(dst, vx, vy, rank, root, obb);
            } else if (!w.rv_lean || (meta & kStepKeep)) {
                RepVal o;
                o.mx = vx;
                o.my = vy;
                o.rank = rank;
                o.root = root;
                o.bb = obb;
                o.pad0 = o.pad1 = 0;
                *dst = o;
            }
        }
        __builtin_amdgcn_s_waitcnt(0xc07f);  // ob reads done before the next chunk overwrites it
        __builtin_amdgcn_wave_barrier();
        if (finished) {  // publish the top: records drained, then the state word; continue its waiter
            f_drain();
            int old = 0;
            if (lane == 0) {
                old = __hip_atomic_exchange(state_at(w, lb + top), kFlowDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (t & kFlowLong) atomicAdd(ctl + FC_LDONE, 1);
                fs_add(ctl, FS_LDONE, 1);
                fs_max(ctl, FS_T_LONG, fs_now());
                if (top == 0) fs_max(ctl, FS_T_ROOT, fs_now());
            }
            old = __shfl(old, 0, 64);
            ret = flow_waiter(w, ctl, old);
            return 1;
        }
        if (n < 64) {  // blocked at pb on light child lq: park on it unless it completed meanwhile
            const int pb = q - n;
            if (n == 0 && w.ord[lb + pb + 1] >= d.N) {  // the state at pb + 1 came from an earlier chunk
                const float mx = __shfl(v, 0, 64), my = __shfl(v, 1, 64);
                if (lane == 0)
                    rv_publish(w.Rv + lb + pb + 1, mx, my, (int)(K >> kRankShift), (int)(K & ((1u << kRankShift) - 1)),
                               bb);
            }
            int parked = 0;
            if (lane == 0) {
                f_st(curp, pb);
                f_drain();
                const int lq = step_lq(w.In[lb + pb], pb);
                const int s0 = f_ld(state_at(w, lb + lq));
                if (s0 != kFlowDone) parked = atomicCAS(state_at(w, lb + lq), s0, t) == s0;
            }
            parked = __shfl(parked, 0, 64);
            if (parked) {
                if (lane == 0) {
                    fs_add(ctl, FS_LPARKS, 1);
                    if (top == 0) fs_add(ctl, FS_RPARKS, 1);
                }
                ret = -1;
                return 1;
            }
            q = pb;  // completed meanwhile: re-resolve the chunk from the blocked step (the caller refills the stages)
            __builtin_amdgcn_wave_barrier();
            OneRec rec2;
            meta = flow_resolve(w, lb, q - lane, top, &rec2, &lbb, pb);
            buf[cb][lane] = rec2;
            curlk = rec2.lk;
            ++restarts;
            return 2;
        }
        q -= 64;
        cb ^= 1;
        meta = nmeta;
        lbb = nlbb;
        FLOW_PROF_MARK(p_tail);
        buf[cb][lane] = nrec;
        curlk = nrec.lk;
        return 0;
    };
    auto pass3 = [&]() -> int {
        int st = iter(i0, i1, i2, r0, r1, r2);
        if (st) return st;
        st = iter(i1, i2, i0, r1, r2, r0);
        if (st) return st;
        return iter(i2, i0, i1, r2, r0, r1);
    };
    for (;;) {  // the first pass after a (re)start is peeled off the steady loop (see flow_pair)
        int st = pass3();
        while (st == 0) st = pass3();
        if (st == 1) break;
        restart_stages(q);
    }
    tally();
    return ret;
}

constexpr int kFlowChunk = 256;  // initial short tasks a short worker claims per atomic (its lanes take them in turn)
constexpr int kFlowHelp = 64;    // initial short tasks an idle long worker claims (one claim, then back to its queue)

// Short paths, one per lane, until no lane has one: idle lanes take initial tasks from the wave's claimed
// chunk [*cbp, *cep), refilled by one atomic of `chunk` tasks at most `claims` times (-1: until the pool is
// empty; 0: never); a lane whose path completes continues the short path parked on its top, and queues a
// long one (a long worker takes it). inject: a short task handed over by a long path's completion (lane 0
// starts with it). Nothing here waits for another wave: every task a wave holds runs to completion or parks.
__device__ __forceinline__ void flow_short(const Ws& w, int* ctl, unsigned epoch, int inject, int claims, int chunk,
                                           int* cbp, int* cep) {
    const Dims& d = w.d;
    const int lane = threadIdx.x & 63;
    const int ntot = ctl[FC_NT] + ctl[FC_NS];
    int t = (lane == 0) ? inject : -1;  // task word (short: no kFlowLong bit)
    bool fresh = t >= 0;
    int q = 0, f = 0;
    int64_t lb = 0;
    int* curp = nullptr;
    RunState s;
    s.mx = s.my = 0.f;
    s.rank = s.root = 0;
    s.bb.x0 = s.bb.y0 = s.bb.x1 = s.bb.y1 = 0;
    for (int it = 0;; ++it) {
        if (claims != 0 || *cbp < *cep) {
            unsigned long long idle = __ballot(t < 0);
            while (idle) {
                if (*cbp >= *cep) {  // claim the next chunk of the pool
                    if (claims == 0) break;
                    int base = 0;
                    if (lane == 0) base = atomicAdd(ctl + FC_SHORT_NEXT, chunk);
                    base = __shfl(base, 0, 64);
                    if (base >= ntot) {
                        claims = 0;
                        break;
                    }
                    if (claims > 0) --claims;
                    *cbp = base;
                    *cep = base + chunk < ntot ? base + chunk : ntot;
                }
                const int avail = *cep - *cbp;
                const int r = __popcll(idle & ((1ull << lane) - 1));
                if (t < 0 && r < avail) {
                    t = flow_short_task(w, ctl, *cbp + r);
                    fresh = true;
                }
                const int took = __popcll(idle) < avail ? __popcll(idle) : avail;
                *cbp += took;
                idle = __ballot(t < 0);
            }
        }
        if (fresh) {  // a new path on this lane: its cursor and the state below it
            fresh = false;
            f = t / (int)d.N;
            const int j = t - f * (int)d.N;
            curp = w.cur + f * d.N + j;
            q = f_ld(curp);
            lb = f * d.NL;
            flow_start(w, f, q + 1, &s.mx, &s.my, &s.rank, &s.root, &s.bb);
        }
        if (!__ballot(t >= 0)) break;
        if (it >= (1 << 26)) {  // (bounded: never reached by a correct run)
            f_st(ctl + FC_ERR, 1);
            break;
        }
        if (t < 0) continue;
        const StepV in = step_v(w.In[lb + q], q, d.W);
        float wbx = in.wbx, wby = in.wby;
        int lrank = 0, lroot = in.lb;
        B4 lbb;
        if (in.meta & kStepDyn) {
            const int lq = in.lb;
            int st = f_ld(state_at(w, lb + lq));
            if (st != kFlowDone) {  // park on the light child: publish the state below q, the cursor
                if (w.ord[lb + q + 1] >= d.N) rv_publish(w.Rv + lb + q + 1, s.mx, s.my, s.rank, s.root, s.bb);
                f_st(curp, q);
                f_drain();
                st = f_ld(state_at(w, lb + lq));
                if (st != kFlowDone && atomicCAS(state_at(w, lb + lq), st, t) == st) {
                    t = -1;
                    continue;
                }
            }
            const RepVal lv = rv_fetch(w.Rv + lb + lq);
            wbx = lv.mx * (float)in.la;
            wby = lv.my * (float)in.la;
            lrank = lv.rank;
            lroot = lv.root;
            lbb = lv.bb;
        } else {
            lbb.x0 = lbb.x1 = (int16_t)(in.la & 0xffff);
            lbb.y0 = lbb.y1 = (int16_t)(in.la >> 16);
        }
        step_merge(s, in.fs, wbx, wby, in.r, in.meta, lrank, lroot, lbb);
        if (in.meta & kStepTop) {  // path complete: publish its top, then continue its waiter
            rv_publish(w.Rv + lb + q, s.mx, s.my, s.rank, s.root, s.bb);
            f_drain();
            const int old = flow_waiter(
                w, ctl, __hip_atomic_exchange(state_at(w, lb + q), kFlowDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            t = -1;
            if (old >= 0) {
                if (old & kFlowLong) {
                    flow_push(w, ctl, epoch, old);
                    fs_add(ctl, FS_PUSH, 1);
                } else {
                    t = old;
                    fresh = true;
                }
            }
            continue;
        }
        if (!w.rv_lean || (in.meta & kStepKeep)) {
            RepVal o;
            o.mx = s.mx;
            o.my = s.my;
            o.rank = s.rank;
            o.root = s.root;
            o.bb = s.bb;
            o.pad0 = o.pad1 = 0;
            w.Rv[lb + q] = o;
        }
        --q;
    }
}

// A long worker's next task: the initial long pool first, then a ticket of the long-path queue, whose slot
// its pusher fills (tickets are taken only while pushes are pending, so there is no atomic herd on the head,
// and at most the racing workers' tickets run ahead of the pushes). A worker whose ticket's slot is not filled
// yet, or that has no ticket, helps with the initial short pool while it is not empty (kFlowHelpTask; it keeps
// its ticket, *ticket, across the help). So a long worker never waits for work that no running wave holds:
// while the short pool has tasks it runs them itself, and once it is empty every unfinished task is held by a
// running wave or parked on one — the replay completes whether the short workers' launch runs beside this
// one, before it or after it (tests/test_gpu_flow_order.py).
// -1: every long path completed, or a bounded wait gave up (C_FLOWERR). A slot is accepted only with this
// launch's tag and a long task word of the batch: slots never written in this launch hold Borůvka minima
// or older tags, which neither passes (kFlowEpochs < the high word of any weight the MST stores there,
// DESIGN.md §6a).
constexpr unsigned kFlowEpochs = 0xFFFFF;
constexpr int kFlowHelpTask = -2;  // flow_next_long: no long task now, the short pool has tasks
__device__ inline int flow_next_long(const Ws& w, int* ctl, unsigned epoch, int nl, int* ticket) {
    const int lane = threadIdx.x & 63;
    int t = -1, tk = *ticket;
    if (lane == 0) {
        const int np = ctl[FC_NLPOOL];
        const int ntot = ctl[FC_NT] + ctl[FC_NS];
        while (tk < 0 && t < 0 && f_poll(ctl + FC_LONG_NEXT) < np) {
            const int i = atomicAdd(ctl + FC_LONG_NEXT, 1);
            if (i < np) t = flow_long_task(w, ctl, i);
        }
        const long long nframe = w.d.N;
        for (int spin = 0; t < 0; ++spin) {
            if (spin >= (1 << 26)) {
                f_st(ctl + FC_ERR, 1);
                break;
            }
            if (tk < 0) {
                if (f_poll(ctl + FC_LDONE) >= nl) break;  // every long path completed: nothing more will come
                if (f_poll(ctl + FC_QHEAD) < f_poll(ctl + FC_QTAIL)) {
                    tk = atomicAdd(ctl + FC_QHEAD, 1);
                    if (tk >= ctl[FC_QCAP]) {  // (never: pushes stay below the capacity)
                        f_st(ctl + FC_ERR, 1);
                        tk = -1;
                        break;
                    }
                    continue;
                }
                if (f_poll(ctl + FC_SHORT_NEXT) < ntot) {
                    t = kFlowHelpTask;
                    break;
                }
                __builtin_amdgcn_s_sleep(32);
                continue;
            }
            const unsigned long long v = f_poll64(w.bw + tk);
            const int c = (int)(unsigned)v;
            if ((unsigned)(v >> 32) == epoch && c >= 0 && (c & kFlowLong) && (long long)(c & kFlowIdMask) < nframe * w.d.B) {
                t = c;
                tk = -1;
                break;
            }
            if ((spin & 15) == 15) {
                if (f_poll(ctl + FC_LDONE) >= nl) {  // a ticket ahead of the last push: never filled
                    tk = -1;
                    break;
                }
                if (f_poll(ctl + FC_SHORT_NEXT) < ntot) {  // the push may need short work: help, keep the ticket
                    t = kFlowHelpTask;
                    break;
                }
            }
            __builtin_amdgcn_s_sleep(16);
        }
    }
    *ticket = __shfl(tk, 0, 64);
    return __shfl(t, 0, 64);
}

// The batch's whole replay, as two persistent launches whose waves work independently (no workgroup
// barrier), packed kW to a workgroup so that they hold few CUs: while they run, the graph stage of the
// next batches (k_krt_fused takes whole CUs) keeps the rest of the chip. Both run at once, the long
// workers on a stream of their own (HipBackend::replay_flow).
//   kLong = false — short workers (8 waves per workgroup): rounds of short paths from the initial pool
//     until it is empty and their lanes are done. A short path parked on a path that completes later
//     is continued by that path's completer; a long path parked on a short one is queued by the lane
//     that completes it.
//   kLong = true — long workers (4 waves per workgroup, one per SIMD, first in its arbitration): long
//     paths from the initial pool (every frame's root chain first), then queue tickets, following their
//     completions' long waiters, and a short waiter as a one-lane short round; they leave when every
//     long path completed.
// Measured (112 frames, 1080p, tools/flow_stats.py, serial): short paths done at 26.7 ms, the last
// chain at 42.4 ms; same-box bench 1,518-1,540 Mpixels/s with 128 long and 2,048 short workers.
template <bool kLong, int kW>
__global__ __launch_bounds__(64 * kW) void k_replay_flow(Ws w, int* ctl, unsigned epoch, int keyfast) {
    __shared__ OneRec buf[kLong ? kW : 1][2][64];
    __shared__ __attribute__((aligned(16))) OneOut ob[kLong ? kW : 1][128];
    const int lane = threadIdx.x & 63;
    const int wv = kLong ? (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) : 0;
    const int nl = ctl[FC_NL];
    int cb = 0, ce = 0;  // this wave's claimed, not yet started initial short tasks
    if (lane == 0) fs_min(ctl, FS_T0, fs_now());
    if constexpr (kLong) {
        __builtin_amdgcn_s_setprio(3);  // the chains go first in their SIMD's arbitration
        int ticket = -1;  // a long-path queue ticket whose slot is not filled yet (kept across help rounds)
        for (int it = 0; it < (1 << 26); ++it) {
            int t = flow_next_long(w, ctl, epoch, nl, &ticket);
            if (t == kFlowHelpTask) {  // idle: one claim of the initial short pool, at the short workers' priority
                __builtin_amdgcn_s_setprio(0);
                flow_short(w, ctl, epoch, -1, 1, kFlowHelp, &cb, &ce);
                __builtin_amdgcn_s_setprio(3);
                continue;
            }
            if (t < 0) break;
            const unsigned long long t1 = fs_now();
            while (t >= 0) {
                if (lane == 0) fs_add(ctl, FS_LRUNS, 1);
                const int nx = flow_long(w, ctl, t, buf[wv], ob[wv], keyfast);
                if (nx >= 0 && !(nx & kFlowLong)) {  // a short waiter: a one-lane short round (and its waiters)
                    if (lane == 0) fs_add(ctl, FS_INJECT, 1);
                    flow_short(w, ctl, epoch, nx, 0, 0, &cb, &ce);
                    break;
                }
                t = nx;
            }
            if (lane == 0) fs_add(ctl, FS_LTICKS, fs_now() - t1);
        }
    } else {
        const unsigned long long t1 = fs_now();
        flow_short(w, ctl, epoch, -1, -1, kFlowChunk, &cb, &ce);
        if (lane == 0) {
            fs_add(ctl, FS_SROUNDS, 1);
            fs_add(ctl, FS_STICKS, fs_now() - t1);
            fs_max(ctl, FS_T_SHORT, fs_now());
        }
    }
    if (lane == 0) fs_max(ctl, FS_T_EXIT, fs_now());
}
// ---------------------------------------------------------------------------------------------
// Long paths by a pair of waves (k_replay_flow_pair). A long path's time is its chain: per 64-step chunk the
// steps (~21 ns each) and, on one wave, the chunk's tail (bbox prefix, record stores, hand-over) and the next
// chunk's resolve (its global loads) — ~1.1 µs a chunk, 17 ns a step more (profiles/r04/anatomy: p_tail
// 30.5 + p_next 30.6 of 157 wave-ms at 4K). One wave issues at most one instruction per four cycles, so the
// tail cannot hide in the chain's idle cycles: it needs a second wave. Here wave C carries the chain alone
// (chain_chunk over LDS records) and wave H, on another SIMD, does everything else one chunk apart: while C
// steps chunk i, H builds chunk i + 1 into the other LDS slot (the three-stage resolve of flow_long) and finishes
// chunk i - 1 (bbox prefix, records); two workgroup barriers per chunk hand the slots over. A chunk that
// completes the path or blocks on an incomplete light child is finished by H at once (C waits), which then
// publishes the top or parks exactly as flow_long does. Task control (queue tickets, help rounds, injected
// short waiters) is H's; C follows the commands H leaves in LDS.
// ---------------------------------------------------------------------------------------------
struct PairShared {
    OneRec buf[2][64];  // step records of the chunk in each slot (H writes, C reads)
    OneOut ob[2][128];  // C's outputs per slot: {v, K} per step, or two rows of 64 values (constant-key)
    int n[2];           // H → C: steps of the chunk in the slot
    int fin[2];         // H → C: the chunk ends the path (its top); with n < 64 a chunk ends the run (blocked)
    unsigned maxlk[2];  // H → C: the largest light key among them (the constant-key test)
    int fast[2];        // C → H: the slot ran as a constant-key chunk ...
    unsigned k0[2];     // C → H: ... with this key
    float sv[2];        // C → H: the carried means after C's last chunk
    unsigned sk;        // C → H: the carried key
    float iv[2];        // H → C: the state at a (re)start
    unsigned ik;
    int cmd;            // H → C: the slot to run next, or kPairEnd
    int ret;            // H → both: the ended task's waiter (or -1)
    int task;           // H → both: the worker's next task word (kernel loop)
};
constexpr int kPairEnd = -1;
constexpr int kPairFrames = 8;  // batches of at most this many frames run their long paths on wave pairs

// the chunk descriptor of a resolved chunk (one lane per step): steps n until the first blocked step or
// through the path's top (finished), and the largest light key among them
__device__ inline int pair_desc(int meta, unsigned lk, bool* fin, unsigned* maxlk) {
    const int lane = threadIdx.x & 63;
    const unsigned long long blocked = __ballot(!(meta & kLongOk));
    const unsigned long long tops = __ballot((meta & kLongOk) && (meta & kStepTop));
    const int fb = blocked ? __ffsll((long long)blocked) - 1 : 64;
    const int ft = tops ? __ffsll((long long)tops) - 1 : 64;
    *fin = ft < fb;
    const int n = *fin ? ft + 1 : fb;
    *maxlk = wave_reduce(lane < n ? lk : 0u, [](unsigned x, unsigned y) { return x > y ? x : y; });
    return n;
}

// A long path (task word t) on the pair, from its cursor; both waves call it (role 0 = H, 1 = C) and both
// return the task word of the parent path parked on its top (to run next), or -1. Per chunk both waves pass
// two workgroup barriers: after the concurrent phase (C's steps of slot s ∥ H's build of the next chunk into
// slot s ^ 1 and tail of the previous chunk) and after H's decision (the slot C runs next, or the end).
__device__ int flow_pair(const Ws& w, int* ctl, int t, PairShared& sh, int keyfast, int role) {
    const Dims& d = w.d;
    const int lane = threadIdx.x & 63;
    const int h = lane & 1;
    const int g = t & kFlowIdMask;
    const int f = g / (int)d.N, j = g - f * (int)d.N;
    int* curp = w.cur + f * d.N + j;
    const int top = w.ptop[f * d.N + j];
    const int64_t lb = f * d.NL;
#ifdef DOFS_FLOW_PROF
    // measurement build: C's steps (p_steps) and its time between chunks (p_tail: barriers, H's decisions);
    // H's concurrent work per chunk (p_next: the next chunk's build and the previous one's tail)
    unsigned long long p_steps = 0, p_tail = 0, p_next = 0, p_skip = 0, p_cwait = 0, p_hwait = 0, p_t = wall_clock64();
#endif
    if (role == 1) {  // ---- C: the chain of every chunk H hands over ----
        __syncthreads();  // H's setup
        if (sh.cmd == kPairEnd) {
            __syncthreads();
            return -1;
        }
        float v = sh.iv[h];
        unsigned K = sh.ik, kfast = 0;
        int sl = 0;
        for (;;) {
            const int n = sh.n[sl];
            const bool cont = n == 64 && !sh.fin[sl];
            const unsigned krank = K & ~((1u << kRankShift) - 1);
            const bool fastc = keyfast && sh.maxlk[sl] < krank;
            const unsigned kstart = K;
            FLOW_PROF_MARK(p_tail);
            chain_chunk(sh.buf[sl], sh.ob[sl], n, fastc, h, v, K);
            FLOW_PROF_MARK(p_steps);
            kfast += fastc ? 1 : 0;
            if (lane == 0) {
                sh.fast[sl] = fastc ? 1 : 0;
                sh.k0[sl] = kstart;
                sh.sk = K;
            }
            if (lane < 2) sh.sv[lane] = v;
            FLOW_PROF_MARK(p_tail);
            __syncthreads();  // the chunk's outputs to H; H has built the next chunk into the other slot
            FLOW_PROF_MARK(p_cwait);
            if (cont) {  // H continues too (it decided from the same descriptor)
                sl ^= 1;
                continue;
            }
            __syncthreads();  // H's decision: the end, or a re-resolved chunk
            if (sh.cmd == kPairEnd) break;
            sl = sh.cmd;
        }
        const int ret = sh.ret;
        if (lane == 0) {
            fs_add(ctl, FS_KFAST, kfast);
#ifdef DOFS_FLOW_PROF
            fs_add(ctl, FS_P_STEPS, p_steps);
            fs_add(ctl, FS_P_TAIL, p_tail);
            fs_add(ctl, FS_P_CWAIT, p_cwait);
#endif
        }
        __syncthreads();  // both read cmd and ret before H may write the next task's words
        return ret;
    }
    // ---- H: everything but the chain ----
    // the chunk in slot s (cursor qs): its records' metas, light boxes and descriptor; the pending tail of the
    // chunk before it (slot p); the carried box; the resolve stages (in named registers)
    int s = 0, qs = f_ld(curp), meta_s = 0, n_s = 0;
    bool fin_s = false;
    B4 lbb_s, bb;
    bool havep = false;
    int p = 0, qp = 0, metap = 0;
    B4 lbbp;
    unsigned chunks = 0, steps = 0, restarts = 1;
    int ret = -1;
    // the resolve stages in named registers rotated by unrolling (no register copies: a copy of a register
    // whose load is in flight waits for it — the rotating form exposed a round trip per chunk). Stage k of
    // the chunk built now: StepIn records in1 / in2 / in3 (chunks qs - 64, - 128, - 192), state words rdy1 /
    // rdy2, and rv, the light records of chunk qs - 64; i0 .. i2 and r0 .. r2 hold them in rotation.
    StepIn i0, i1, i2;
    int r0, r1, r2;
    RepVal rv;
    // (re)fill the stages for the chunks after cursor q, synchronously: the explicit wait leaves no load in
    // flight at the loop head, where this path meets the back edge (else the compiler's waits at the head
    // merge both paths' pending loads and expose a round trip per pass)
    auto restart_stages = [&](int q) {
        i0 = pipe_in(w, lb, q - 64 - lane, top);
        i1 = pipe_in(w, lb, q - 128 - lane, top);
        i2 = pipe_in(w, lb, q - 192 - lane, top);
        r0 = pipe_rdy(w, lb, i0, q - 64 - lane, top);
        r1 = pipe_rdy(w, lb, i1, q - 128 - lane, top);
        rv = pipe_rv(w, lb, i0, r0, q - 64 - lane, top);
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    };
    {
        float mx, my;
        int rank, root;
        flow_start(w, f, qs + 1, &mx, &my, &rank, &root, &bb);
        if (lane == 0) {
            sh.iv[0] = mx;
            sh.iv[1] = my;
            sh.ik = rk_pack(rank, root);
        }
        OneRec rec;
        meta_s = flow_resolve(w, lb, qs - lane, top, &rec, &lbb_s);
        sh.buf[0][lane] = rec;
        unsigned mk;
        n_s = pair_desc(meta_s, rec.lk, &fin_s, &mk);
        if (lane == 0) {
            sh.n[0] = n_s;
            sh.fin[0] = fin_s ? 1 : 0;
            sh.maxlk[0] = mk;
            sh.cmd = qs < top ? kPairEnd : 0;  // (never: a task is handed out only while its path is not complete)
            sh.ret = -1;
        }
        restart_stages(qs);
    }
    __syncthreads();
    if (sh.cmd == kPairEnd) {
        __syncthreads();
        return -1;
    }
    // H: the tail of the chunk in slot sl (cursor qc, n steps): the bbox prefix joined with the carried box,
    // then the records the results read; the chunk's last record published if it ends the path or blocks
    auto tail = [&](int sl, int qc, int n, bool last, const B4& lb4, int meta) {
        B4 x = lb4;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const B4 y = bb_shfl_up(x, o);
            if (lane >= o) x = bb_join(x, y);
        }
        x = bb_join(x, bb);
        const int src = n > 0 ? n - 1 : 0;
        const int lo = __shfl((int)((unsigned short)x.x0 | ((unsigned)(unsigned short)x.y0 << 16)), src, 64);
        const int hi = __shfl((int)((unsigned short)x.x1 | ((unsigned)(unsigned short)x.y1 << 16)), src, 64);
        if (n > 0) {
            bb.x0 = (int16_t)(lo & 0xffff);
            bb.y0 = (int16_t)(lo >> 16);
            bb.x1 = (int16_t)(hi & 0xffff);
            bb.y1 = (int16_t)(hi >> 16);
        }
        if (lane < n) {
            const bool fastc = sh.fast[sl] != 0;
            const float* fv = reinterpret_cast<const float*>(sh.ob[sl]);
            const OneOut sx = sh.ob[sl][2 * lane], sy = sh.ob[sl][2 * lane + 1];
            const float vx = fastc ? fv[lane] : sx.v, vy = fastc ? fv[64 + lane] : sy.v;
            const unsigned kk = fastc ? sh.k0[sl] : sx.k;
            const int rank = (int)(kk >> kRankShift), root = (int)(kk & ((1u << kRankShift) - 1));
            RepVal* dst = w.Rv + lb + qc - lane;
            if (lane == n - 1 && last) {
                rv_publish(dst, vx, vy, rank, root, x);
            } else if (!w.rv_lean || (meta & kStepKeep)) {
                RepVal o;
                o.mx = vx;
                o.my = vy;
                o.rank = rank;
                o.root = root;
                o.bb = x;
                o.pad0 = o.pad1 = 0;
                *dst = o;
            }
        }
    };
    // one chunk of H: 0 = continue (slot s advanced), 1 = the task ended (ret), 2 = restarted (canonical stages)
    auto iter = [&](StepIn& in1, StepIn& in2, StepIn& in3, int& rdy1, int& rdy2, int& rdy3) -> int {
        // concurrent phase: the next chunk into the other slot, whether or not this one continues (no branch
        // around the stage loads), and the pending tail
        FLOW_PROF_MARK(p_skip);
        OneRec nrec;
        B4 nlbb;
        const int nmeta = pipe_build(w, in1, rdy1, rv, qs - 64 - lane, top, &nrec, &nlbb);
        rv = pipe_rv(w, lb, in2, rdy2, qs - 128 - lane, top);  // issued now, used a chunk later
        rdy3 = pipe_rdy(w, lb, in3, qs - 192 - lane, top);
        in1 = pipe_in(w, lb, qs - 256 - lane, top);  // (in1 was consumed by pipe_build)
        sh.buf[s ^ 1][lane] = nrec;
        unsigned mk;
        bool nfin;
        const int nn = pair_desc(nmeta, nrec.lk, &nfin, &mk);
        if (lane == 0) {
            sh.n[s ^ 1] = nn;
            sh.fin[s ^ 1] = nfin ? 1 : 0;
            sh.maxlk[s ^ 1] = mk;
        }
        if (havep) {
            tail(p, qp, 64, false, lbbp, metap);
            havep = false;
        }
        FLOW_PROF_MARK(p_next);
        __syncthreads();  // C's outputs of slot s
        FLOW_PROF_MARK(p_hwait);
        // decision: continue, or finish the chunk now (the path completes or blocks)
        int cmd = 0, st = 0;
        ++chunks;
        steps += n_s;
        if (n_s == 64 && !fin_s) {  // continue with the next slot; this chunk's tail overlaps C's next chunk
            havep = true;
            p = s;
            qp = qs;
            metap = meta_s;
            lbbp = lbb_s;
            s ^= 1;
            qs -= 64;
            meta_s = nmeta;
            lbb_s = nlbb;
            n_s = nn;
            fin_s = nfin;
            return 0;  // (C reads the same descriptor: no second barrier)
        } else {
            tail(s, qs, n_s, true, lbb_s, meta_s);
            if (fin_s) {  // publish the top: records drained, then the state word; its waiter runs next
                f_drain();
                int old = 0;
                if (lane == 0) {
                    old = __hip_atomic_exchange(state_at(w, lb + top), kFlowDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (t & kFlowLong) atomicAdd(ctl + FC_LDONE, 1);
                    fs_add(ctl, FS_LDONE, 1);
                    fs_max(ctl, FS_T_LONG, fs_now());
                    if (top == 0) fs_max(ctl, FS_T_ROOT, fs_now());
                }
                old = __shfl(old, 0, 64);
                ret = flow_waiter(w, ctl, old);
                cmd = kPairEnd;
                st = 1;
            } else {  // blocked at pb on light child lq: park on it unless it completed meanwhile
                const int pb = qs - n_s;
                if (n_s == 0 && w.ord[lb + pb + 1] >= d.N && lane == 0)  // the state at pb + 1: C's carried one
                    rv_publish(w.Rv + lb + pb + 1, sh.sv[0], sh.sv[1], (int)(sh.sk >> kRankShift),
                               (int)(sh.sk & ((1u << kRankShift) - 1)), bb);
                int parked = 0;
                if (lane == 0) {
                    f_st(curp, pb);
                    f_drain();
                    const int lq = step_lq(w.In[lb + pb], pb);
                    const int s0 = f_ld(state_at(w, lb + lq));
                    if (s0 != kFlowDone) parked = atomicCAS(state_at(w, lb + lq), s0, t) == s0;
                }
                parked = __shfl(parked, 0, 64);
                if (parked) {
                    if (lane == 0) {
                        fs_add(ctl, FS_LPARKS, 1);
                        if (top == 0) fs_add(ctl, FS_RPARKS, 1);
                    }
                    ret = -1;
                    cmd = kPairEnd;
                    st = 1;
                } else {  // completed meanwhile: re-resolve the chunk from the blocked step
                    qs = pb;
                    s ^= 1;
                    OneRec rec;
                    meta_s = flow_resolve(w, lb, qs - lane, top, &rec, &lbb_s, pb);
                    sh.buf[s][lane] = rec;
                    n_s = pair_desc(meta_s, rec.lk, &fin_s, &mk);
                    if (lane == 0) {
                        sh.n[s] = n_s;
                        sh.fin[s] = fin_s ? 1 : 0;
                        sh.maxlk[s] = mk;
                    }
                    ++restarts;
                    cmd = s;
                    st = 2;  // (the caller refills the stages)
                }
            }
        }
        if (lane == 0) {
            sh.cmd = cmd;
            sh.ret = ret;
        }
        __syncthreads();  // the decision to C
        return st;
    };
    // three chunks per pass: the stages rotate through i0 .. i2 and r0 .. r2. The first pass after a (re)start
    // is peeled off the steady loop, whose head is then reached only after a third chunk (the compiler's waits
    // at a loop head merge its predecessors' loads in flight: a restart's would make them all vmcnt(0))
    auto pass3 = [&]() -> int {
        int st = iter(i0, i1, i2, r0, r1, r2);
        if (st) return st;
        st = iter(i1, i2, i0, r1, r2, r0);
        if (st) return st;
        return iter(i2, i0, i1, r2, r0, r1);
    };
    for (;;) {
        int st = pass3();
        while (st == 0) st = pass3();
        if (st == 1) break;
        restart_stages(qs);
    }
    if (lane == 0) {
        fs_add(ctl, FS_LCHUNKS, chunks);
        fs_add(ctl, FS_LSTEPS, steps);
        fs_add(ctl, FS_RESTARTS, restarts);
        if (top == 0) {
            fs_add(ctl, FS_RCHUNKS, chunks);
            fs_add(ctl, FS_RSTEPS, steps);
        }
#ifdef DOFS_FLOW_PROF
        fs_add(ctl, FS_P_NEXT, p_next);
        fs_add(ctl, FS_P_HWAIT, p_hwait);
        (void)p_skip;
        (void)p_cwait;
        (void)p_steps;
        (void)p_tail;
#endif
    }
    __syncthreads();  // both read cmd and ret before H may write the next task's words
    return ret;
}

// Long workers as wave pairs (flow_pair): one workgroup of two waves per worker, H (wave 0) and C (wave 1).
// The task loop of k_replay_flow<true, ...>, with H taking the decisions and both waves helping with the
// short pool when H finds no long task (each wave one claim).
__global__ __launch_bounds__(128) void k_replay_flow_pair(Ws w, int* ctl, unsigned epoch, int keyfast) {
    __shared__ PairShared sh;
    const int lane = threadIdx.x & 63;
    const int role = (int)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int nl = ctl[FC_NL];
    int cb = 0, ce = 0;
    int ticket = -1;
    if (lane == 0) fs_min(ctl, FS_T0, fs_now());
    __builtin_amdgcn_s_setprio(3);
    for (int it = 0; it < (1 << 26); ++it) {
        if (role == 0) {
            const int t0 = flow_next_long(w, ctl, epoch, nl, &ticket);
            if (lane == 0) sh.task = t0;
        }
        __syncthreads();
        int t = sh.task;
        if (t == -1) break;
        if (t == kFlowHelpTask) {  // one claim of the initial short pool per wave, at the short workers' priority
            __builtin_amdgcn_s_setprio(0);
            flow_short(w, ctl, epoch, -1, 1, kFlowHelp, &cb, &ce);
            __builtin_amdgcn_s_setprio(3);
            __syncthreads();
            continue;
        }
        const unsigned long long t1 = fs_now();
        while (t >= 0) {
            if (role == 0 && lane == 0) fs_add(ctl, FS_LRUNS, 1);
            const int nx = flow_pair(w, ctl, t, sh, keyfast, role);
            if (nx >= 0 && !(nx & kFlowLong)) {  // a short waiter: a one-lane short round on H (and its waiters)
                if (role == 0) {
                    if (lane == 0) fs_add(ctl, FS_INJECT, 1);
                    flow_short(w, ctl, epoch, nx, 0, 0, &cb, &ce);
                }
                break;
            }
            t = nx;
        }
        __syncthreads();
        if (role == 0 && lane == 0) fs_add(ctl, FS_LTICKS, fs_now() - t1);
    }
    if (lane == 0) fs_max(ctl, FS_T_EXIT, fs_now());
}

#ifndef DOFS_FLOW_SHORT_W
#define DOFS_FLOW_SHORT_W 8
#endif
constexpr int kFlowShortW = DOFS_FLOW_SHORT_W;  // waves per short-worker workgroup
constexpr int kFlowLongW = 4;    // waves per long-worker workgroup (one per SIMD)

// counter C_FLOWERR of frame 0 = a bounded wait of the launch gave up (dofs_batch_counters); force: a test
// of the error's path through the accessors (dofs_debug_flow_giveup), the replay itself is complete
__global__ void k_flow_report(Ws w, const int* ctl, int force) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && (ctl[FC_ERR] || force)) w.C(0)[C_FLOWERR] = kErrGiveUp;
}
inline int g_flow_giveup = 0;  // host: dofs_debug_flow_giveup (test only)
// test only (dofs_debug_bad_root): a root outside the frame written into each frame's last merge record (the
// KRT root: size H*W, a scoring candidate's record) after the replay, as a stale or torn record would hold one
__global__ void k_bad_root(Ws w) {
    if (blockIdx.x != 0 || w.d.M <= 0) return;
    for (int f = threadIdx.x; f < w.d.B; f += blockDim.x) {
        const int64_t lb = f * w.d.NL;
        w.Rv[lb + w.pre[lb + w.d.N + w.d.M - 1]].root = (int)w.d.N + 7;
    }
}
inline int g_bad_root = 0;  // host: dofs_debug_bad_root (test only)

}  // namespace dofs
