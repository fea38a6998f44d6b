"""Per-queue busy time and idle gaps of a rocprofv3 kernel trace (run_kernel_trace.csv): how much of
the wall time each stream's kernels cover, and how much of it both streams run at once."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
t_lo = min(int(r["Start_Timestamp"]) for r in rows)
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # seconds to drop at the start (warmup)
by = {}
for r in rows:
    s, e = int(r["Start_Timestamp"]) - t_lo, int(r["End_Timestamp"]) - t_lo
    if s < skip * 1e9:
        continue
    by.setdefault(r[key], []).append((s, e, r["Kernel_Name"][:60]))


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e, *_ in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


allv = [x for v in by.values() for x in v]
lo, hi = min(x[0] for x in allv), max(x[1] for x in allv)
print(f"window {(hi - lo) / 1e6:.1f} ms, {len(allv)} kernels")
unions = {}
for q, v in sorted(by.items()):
    u = union(v)
    unions[q] = u
    busy = sum(e - s for s, e in u)
    gaps = sorted(((u[i + 1][0] - u[i][1], u[i][1], v) for i in range(len(u) - 1)), reverse=True)[:5]
    print(f"{key} {q}: {len(v)} kernels, busy {busy / 1e6:.1f} ms ({100 * busy / (hi - lo):.1f} %), "
          f"largest gaps (ms): {[round(g[0] / 1e6, 2) for g in gaps]}")
qs = list(unions)
if len(qs) >= 2:
    ev = []
    for q in qs:
        for s, e in unions[q]:
            ev += [(s, 1), (e, -1)]
    ev.sort()
    cur, last, both, none = 0, lo, 0, 0
    for t, d in ev:
        if cur >= 2:
            both += t - last
        if cur == 0:
            none += t - last
        cur += d
        last = t
    print(f"two or more streams busy: {both / 1e6:.1f} ms; no stream busy: {none / 1e6:.1f} ms")
