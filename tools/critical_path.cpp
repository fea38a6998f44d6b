// critical_path.cpp — the replay's dependency chain of one frame, from its merge stream.
//
// Input (stdin, binary): int64 N, then N-1 pairs (int32 start, int32 end) — the endpoints of every merge in
// Kruskal order (dofs_events' start / end). Builds the Kruskal reconstruction tree (children = the two
// components' KRT nodes, heavy = the start side's unless the end side is larger — the product's rule,
// deep_parent), its heavy paths, and evaluates the dataflow replay (dofs_dataflow.h) with unlimited workers:
//   a step at merge x runs after the step below it on its path and after its light child's path completed;
//   it costs c_long on a path of >= long_path merges (a wave's chunk loop) and c_short on a shorter one (one
//   lane), plus c_wake when the path had parked on the light child (waiting for it).
// Output (stdout, JSON): the KRT height in merges (the chain with every step costing 1 and no wake-ups), the
// root heavy path's length, the modelled critical-path time for the costs given, and the critical path's
// composition (steps on long paths, on short paths, wake-ups) traced back from the root.
// Usage: critical_path c_long_ns c_short_ns c_wake_ns long_path < pairs.bin
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

static int find(std::vector<int>& p, int x) {
    while (p[x] != x) {
        p[x] = p[p[x]];
        x = p[x];
    }
    return x;
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: critical_path c_long_ns c_short_ns c_wake_ns long_path < pairs.bin\n");
        return 2;
    }
    const double cl = atof(argv[1]), cs = atof(argv[2]), cw = atof(argv[3]);
    const int long_path = atoi(argv[4]);
    int64_t N = 0;
    if (fread(&N, 8, 1, stdin) != 1 || N < 2) return 2;
    const int64_t M = N - 1, NL = N + M;
    std::vector<int> se(2 * M);
    if (fread(se.data(), 4, 2 * M, stdin) != (size_t)(2 * M)) return 2;
    // KRT: node ids 0..N-1 pixels, N + k merge k
    std::vector<int> par(N), lab(N), heavy(M), light(M);
    std::vector<int64_t> size(NL, 1);
    for (int64_t i = 0; i < N; ++i) par[i] = lab[i] = (int)i;
    for (int64_t k = 0; k < M; ++k) {
        const int ra = find(par, se[2 * k]), rb = find(par, se[2 * k + 1]);
        if (ra == rb) {
            fprintf(stderr, "merge %lld joins one component\n", (long long)k);
            return 3;
        }
        const int a = lab[ra], b = lab[rb];
        const bool lightB = size[a] >= size[b];
        heavy[k] = lightB ? a : b;
        light[k] = lightB ? b : a;
        size[N + k] = size[a] + size[b];
        par[rb] = ra;
        lab[ra] = (int)(N + k);
    }
    // path of each merge: top = a merge that is the root or some merge's light child; path length = merges
    // from the top down the heavy children. Walk from each top (children have lower ranks than parents).
    std::vector<int> plen(M, 0);  // path length, stored at every merge of the path
    std::vector<char> is_top(M, 0);
    is_top[M - 1] = 1;
    for (int64_t k = 0; k < M; ++k)
        if (light[k] >= N) is_top[light[k] - N] = 1;
    for (int64_t k = M - 1; k >= 0; --k) {
        if (!is_top[k]) continue;
        int len = 0;
        for (int x = (int)(N + k); x >= N; x = heavy[x - N]) ++len;
        for (int x = (int)(N + k); x >= N; x = heavy[x - N]) plen[x - N] = len;
    }
    // unlimited-worker schedule in rank order (every child precedes its parent)
    std::vector<double> t(NL, 0.0);  // completion time of node x's step (pixels: 0)
    std::vector<int64_t> h(NL, 0);   // unit-cost chain length (the KRT height below x)
    std::vector<char> via_light(M, 0), woke(M, 0);
    for (int64_t k = 0; k < M; ++k) {
        const int a = heavy[k], b = light[k];
        const bool lng = plen[k] >= long_path;
        const double c = lng ? cl : cs;
        double start = t[a];
        bool wk = false;
        if (t[b] > start) {  // the light child completes after the path reached it: park, wake
            start = t[b] + cw;
            wk = true;
        }
        t[N + k] = start + c;
        via_light[k] = t[b] > t[a];
        woke[k] = wk;
        h[N + k] = 1 + (h[a] > h[b] ? h[a] : h[b]);
    }
    // trace the critical path back from the root: at each merge, the later of its two inputs
    int64_t steps_long = 0, steps_short = 0, wakes = 0, paths = 0;
    int x = (int)(NL - 1);
    int cur_top_len = -1;
    while (x >= N) {
        const int64_t k = x - N;
        if (plen[k] >= long_path)
            ++steps_long;
        else
            ++steps_short;
        if (plen[k] != cur_top_len) {
            ++paths;
            cur_top_len = plen[k];
        }
        if (woke[k]) ++wakes;
        x = via_light[k] ? light[k] : heavy[k];
        if (via_light[k]) cur_top_len = -1;
    }
    int64_t root_len = plen[M - 1];
    int64_t nlong = 0, long_merges = 0;
    for (int64_t k = 0; k < M; ++k)
        if (is_top[k] && plen[k] >= long_path) {
            ++nlong;
            long_merges += plen[k];
        }
    printf("{\"N\": %lld, \"krt_height\": %lld, \"root_path\": %lld, \"long_paths\": %lld, \"long_path_merges\": %lld, "
           "\"model_ms\": %.4f, \"costs_ns\": {\"long_step\": %g, \"short_step\": %g, \"wake\": %g}, \"long_path\": %d, "
           "\"critical\": {\"steps_long\": %lld, \"steps_short\": %lld, \"wakes\": %lld, \"paths\": %lld}}\n",
           (long long)N, (long long)h[NL - 1], (long long)root_len, (long long)nlong, (long long)long_merges,
           t[NL - 1] / 1e6, cl, cs, cw, long_path, (long long)steps_long, (long long)steps_short, (long long)wakes,
           (long long)paths);
    return 0;
}
