// Can an agent-scope (sc1) load return a stale copy of a 32-byte sector that another XCD has since
// republished with drained sc1 stores? ("hand-offs of replay records".)
//
// The replay hands records between waves on any XCD: the producer stores a record with write-through
// (sc1) stores, drains them (s_waitcnt vmcnt(0)) and then flips a state word; the consumer reads the state
// word and then the record with sc1 loads. Round 5's explanation of a fault assumed that a consumer-side
// sc1 load made BEFORE the publish (a don't-care load of a not-yet-published record, or a neighbouring
// record of the same sector) leaves a copy of the line in the consumer XCD's L2, which a later sc1 load
// then returns stale. This tool tests exactly that sequence, one trial per fresh 128-byte line:
//   consumer C (one wave, XCD X): (1) first load of word `a` of the line (none / sc1 / plain);
//       (2) optionally an agent-scope CAS on word 4 of the same sector (the park path's CAS);
//       (3) drained, then signals P (sc1 flag store);
//   producer P (one wave, XCD Y): waits for the signal, sc1-stores a new value to word `b`, drains,
//       sc1-stores its flag;
//   C: polls P's flag (sc1 loads), then re-loads word `b` (sc1, or plain for the positive control):
//       stale = the value before P's store.
// A last case has C plain-store a neighbouring word of the same sector before signalling (a 24-byte record's
// neighbour written by another wave), and the host then checks every line in memory: a write-back of C's
// copy of the line must not undo P's bytes (lost = a line whose P word or C word does not hold its value).
// Pairs are (block 2k, 2k+1) (dealt to different XCDs) or (block k, k+8) (the same XCD); every block
// records its XCC id, so each trial is classified by the XCDs it actually ran on. Every wait is bounded
// (a timeout is counted, never a hang). Build: hipcc --offload-arch=gfx950 -O3 -o tools/_build/stale_sector_micro
// tools/stale_sector_micro.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

constexpr int kPairs = 32;
constexpr int kLineInts = 32;   // 128-byte line per trial
constexpr int kFlagInts = 64;   // 256-byte line per flag
constexpr int kSpin = 1 << 22;  // bounded waits

__device__ inline int ld_sc1(const int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline void st_sc1(int* p, int v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ inline void drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ inline int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

struct Cfg {
    int first;    // 0 none, 1 sc1 load, 2 plain load
    int cas;      // 1: agent CAS on word 4 between the first load and the signal
    int a, b;     // word C loads first, word P republishes (same line)
    int reload;   // 1 sc1 re-load, 2 plain re-load (positive control: L1 keeps the line)
    int dist;     // pair distance in blocks: 1 (different XCDs) or 8 (same XCD)
    int cst;      // >= 0: C plain-stores this word of the line before signalling (a neighbour record's store)
};

// out[blk] = XCC id; res[pair * 4 + {0 stale, 1 timeouts, 2 trials}]
__global__ void probe(int* lines, int* flags, int* xcc, int* res, int trials, Cfg c) {
    if (threadIdx.x != 0) return;
    const int b = blockIdx.x;
    const int grp = b / (2 * c.dist), off = b % (2 * c.dist);
    const bool consumer = off < c.dist;
    const int pair = grp * c.dist + (consumer ? off : off - c.dist);
    xcc[b] = xcc_id();
    int* fc = flags + (2 * pair) * kFlagInts;      // C -> P
    int* fp = flags + (2 * pair + 1) * kFlagInts;  // P -> C
    int stale = 0, tmo = 0;
    for (int t = 0; t < trials; ++t) {
        int* line = lines + ((int64_t)pair * trials + t) * kLineInts;
        const int nv = 1000 + t;
        if (consumer) {
            int v0 = 0;
            if (c.first == 1) v0 = ld_sc1(line + c.a);
            if (c.first == 2) v0 = line[c.a];
            drain();
            if (c.cas) atomicCAS(line + 4, -7, -8);  // (fails: word 4 holds 0; still an agent atomic on the sector)
            if (c.cst >= 0) line[c.cst] = 77 + t;
            drain();
            fc[1] = v0;  // keeps the first load live (on the flag's line, never on the probed line)
            st_sc1(fc, t + 1);
            int s = 0;
            while (ld_sc1(fp) != t + 1 && ++s < kSpin) __builtin_amdgcn_s_sleep(1);
            if (s >= kSpin) {
                ++tmo;
                break;
            }
            const int v1 = c.reload == 1 ? ld_sc1(line + c.b) : line[c.b];
            if (v1 != nv) ++stale;
        } else {
            int s = 0;
            while (ld_sc1(fc) != t + 1 && ++s < kSpin) __builtin_amdgcn_s_sleep(1);
            if (s >= kSpin) {
                ++tmo;
                break;
            }
            st_sc1(line + c.b, nv);
            drain();
            st_sc1(fp, t + 1);
            drain();
        }
    }
    if (consumer) {
        res[pair * 4 + 0] = stale;
        res[pair * 4 + 1] += tmo;
        res[pair * 4 + 2] = trials;
    } else {
        res[pair * 4 + 3] = tmo;
    }
}

int main(int argc, char** argv) {
    const int trials = argc > 1 ? atoi(argv[1]) : 2000;
    const size_t line_bytes = (size_t)kPairs * trials * kLineInts * 4;
    int *lines, *flags, *xcc, *res;
    if (hipMalloc(&lines, line_bytes) != hipSuccess) return 1;
    if (hipMalloc(&flags, 2 * kPairs * kFlagInts * 4) != hipSuccess) return 1;
    if (hipMalloc(&xcc, 2 * kPairs * 4) != hipSuccess) return 1;
    if (hipMalloc(&res, kPairs * 4 * 4) != hipSuccess) return 1;
    struct Named {
        const char* name;
        Cfg c;
    };
    const Named cfgs[] = {
        {"no first load, sc1 reload (baseline)", {0, 0, 0, 0, 1, 1, -1}},
        {"sc1 first load of the same word, sc1 reload", {1, 0, 0, 0, 1, 1, -1}},
        {"sc1 first load of the same word, CAS, sc1 reload", {1, 1, 0, 0, 1, 1, -1}},
        {"sc1 load of word 0, P writes word 2 (same sector)", {1, 0, 0, 2, 1, 1, -1}},
        {"sc1 load of word 0, P writes word 8 (next sector, same line)", {1, 0, 0, 8, 1, 1, -1}},
        {"plain first load, sc1 reload", {2, 0, 0, 0, 1, 1, -1}},
        {"plain first load, plain reload (positive control)", {2, 0, 0, 0, 2, 1, -1}},
        {"same XCD: sc1 first load, sc1 reload", {1, 0, 0, 0, 1, 8, -1}},
        {"same XCD: plain first load, plain reload (positive control)", {2, 0, 0, 0, 2, 8, -1}},
        {"plain load of word 0, C plain-stores word 6, P writes word 0 (same sector)", {2, 0, 0, 0, 1, 1, 6}},
        {"sc1 load of word 6, C plain-stores word 6, P writes word 2 (same sector)", {1, 0, 6, 2, 1, 1, 6}},
    };
    std::vector<int> hx(2 * kPairs), hr(kPairs * 4);
    printf("{\"trials_per_pair\": %d, \"pairs\": %d, \"results\": [\n", trials, kPairs);
    for (size_t k = 0; k < sizeof(cfgs) / sizeof(cfgs[0]); ++k) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipMemset(lines, 0, line_bytes);
            (void)hipMemset(flags, 0, 2 * kPairs * kFlagInts * 4);
            (void)hipMemset(res, 0, kPairs * 4 * 4);
            (void)hipDeviceSynchronize();
            hipLaunchKernelGGL(probe, dim3(2 * kPairs), dim3(64), 0, 0, lines, flags, xcc, res, trials, cfgs[k].c);
            if (hipDeviceSynchronize() != hipSuccess) {
                printf("launch failed\n");
                return 1;
            }
            (void)hipMemcpy(hx.data(), xcc, 2 * kPairs * 4, hipMemcpyDeviceToHost);
            (void)hipMemcpy(hr.data(), res, kPairs * 4 * 4, hipMemcpyDeviceToHost);
            long long st_cross = 0, n_cross = 0, st_same = 0, n_same = 0, tmo = 0, lost = 0;
            {  // the lines in memory after the launch: P's word (and C's, where it stored one) hold their values
                std::vector<int> hl(line_bytes / 4);
                (void)hipMemcpy(hl.data(), lines, line_bytes, hipMemcpyDeviceToHost);
                for (int p = 0; p < kPairs; ++p)
                    for (int t = 0; t < trials; ++t) {
                        const int* L = hl.data() + ((size_t)p * trials + t) * kLineInts;
                        if (L[cfgs[k].c.b] != 1000 + t || (cfgs[k].c.cst >= 0 && L[cfgs[k].c.cst] != 77 + t)) ++lost;
                    }
            }
            const int dist = cfgs[k].c.dist;
            for (int p = 0; p < kPairs; ++p) {
                const int grp = p / dist, o = p % dist;
                const int bc = grp * 2 * dist + o, bp = bc + dist;
                const bool same = hx[bc] == hx[bp];
                (same ? st_same : st_cross) += hr[p * 4 + 0];
                (same ? n_same : n_cross) += hr[p * 4 + 2];
                tmo += hr[p * 4 + 1] + hr[p * 4 + 3];
            }
            printf("  {\"case\": \"%s\", \"rep\": %d, \"cross_xcd_trials\": %lld, \"cross_xcd_stale\": %lld, "
                   "\"same_xcd_trials\": %lld, \"same_xcd_stale\": %lld, \"timeouts\": %lld, \"lost_in_memory\": %lld}%s\n",
                   cfgs[k].name, rep, n_cross, st_cross, n_same, st_same, tmo, lost,
                   (k + 1 == sizeof(cfgs) / sizeof(cfgs[0]) && rep == 1) ? "" : ",");
        }
    }
    printf("]}\n");
    return 0;
}
