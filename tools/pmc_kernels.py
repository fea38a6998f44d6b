"""Per-kernel PMC summary of a bench run (rocprofv3 --pmc passes, one counter group per pass).

usage: python tools/pmc_kernels.py OUT_DIR CALIB_JSON K1,K2,... [BATCH] > summary.json

Output: {"batch", "height", "width", "kernels": {name: ...}} — bench.py --pmc reads it (roofline traffic).

OUT_DIR holds the pass directories pmc_fetch/ (FETCH_SIZE), pmc_write/ (WRITE_SIZE), pmc_sq/ (SQ
issue/wait counters) and pmc_tcc/ (L2 hits / misses). For each kernel (functor or kernel name, e.g.
k_krt_fused, KJump) the per-dispatch values are averaged.

Counter semantics, from the calibration of tools/fetch_calib.hip (CALIB_JSON, tools/calib.py, gfx950):
coalesced reads of 4, 8 and 16 B per lane all count exactly half their bytes in FETCH_SIZE (128-B
lines tallied at 64 B), so their HBM bytes are 2 x FETCH_SIZE; a random 4- or 16-B read counts 64 B
(one request); WRITE_SIZE counts coalesced stores exactly and a random 8-B store as 32 B. So
hbm_read_bytes = 2 x FETCH_SIZE for kernels whose reads are coalesced (pattern "stream"), and FETCH_SIZE
(one 64-B request per access, a lower bound) for kernels dominated by random accesses ("random"), and
both bounds for a "mixed" kernel (hbm_read_bounds = [FETCH_SIZE, 2 x FETCH_SIZE]; hbm_read_bytes = the
upper one). A fifth pass, pmc_rdreq/ (TCC_EA0_RDREQ_{32B,64B,128B}_sum), counts the L2's memory-side read
requests by size: read_bytes_by_request_size = 32 R32 + 64 R64 + 128 R128 needs no pattern factor
(tools/calib.py checks it on the calibration kernels) and, when present, is the kernel's read bytes.
"""
import csv
import glob
import json
import os
import sys

# dominant access pattern of each kernel's reads (see the docstring)
PATTERN = {
    "k_boruvka_min": "stream",   # tile label / flow rows, candidate words per pixel
    "k_boruvka_min4": "stream",  # tile label / flow rows (16-B loads), records per tile
    "k_boruvka_recs<false>": "stream",  # records by tile (k_boruvka_pick4)
    "k_boruvka_recs<true>": "stream",   # records by tile (k_boruvka_hookr)
    "KOrd": "stream",            # jump words by node; the ord[] scatter is random 4-B stores
    "k_krt_fused": "random",     # union-find records, label / seed stores
    "k_replay_long1": "stream",  # StepIn / RepVal records by preorder position (64-step chunks)
    "k_replay_flow": "mixed",    # StepIn / RepVal by preorder position (waves: 64-step chunks, coalesced), short
                                 # paths one per lane and light children's records gathered at random
    "KJump": "random",
    "KPathInit": "random",
    "KLift": "random",
    "KFilter": "random",
    "k_pre_sweep": "random",     # jump words of later blocks (gathers); the ord[] scatter
    "k_blur_fused": "stream",    # tile + halo rows of the flow in, the blurred tile out
}


def rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        out.extend(csv.DictReader(open(f)))
    return out


def match(name, k):
    return (f"dofs::{k}(" in name or f"dofs::{k}>" in name or f"::{k}(" in name
            or (k.endswith(">") and f"dofs::{k}(" in name.replace("void ", "")))


# kernels the bench times as ONE probe launch made of several dispatches (HipBackend::replay_flow: the
# long and the short workers side by side): their counters are the sum of the instances' per-dispatch means
INSTANCES = {"k_replay_flow": ["k_replay_flow<true, 4>", "k_replay_flow<false, 8>"]}


def per_dispatch(rs, k):
    """{counter: mean over dispatches of the per-dispatch sum}"""
    if k in INSTANCES:
        tot = {}
        for inst in INSTANCES[k]:
            for c, (m, n) in per_dispatch(rs, inst).items():
                v, n0 = tot.get(c, (0.0, n))
                tot[c] = (v + m, n0)
        return tot
    acc = {}
    for r in rs:
        if not match(r.get("Kernel_Name", ""), k):
            continue
        c = r["Counter_Name"]
        acc.setdefault(c, {}).setdefault(r["Dispatch_Id"], 0.0)
        acc[c][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: (sum(v.values()) / len(v), len(v)) for c, v in acc.items()}


def main():
    out_dir, calib_path, kernels = sys.argv[1], sys.argv[2], sys.argv[3].split(",")
    calib = json.load(open(calib_path)) if os.path.exists(calib_path) else {}
    passes = {p: rows(os.path.join(out_dir, p)) for p in ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_tcc", "pmc_rdreq")}
    if not passes["pmc_fetch"]:  # tools/gpu_ab.sh layout: one directory per counter
        passes["pmc_fetch"] = rows(os.path.join(out_dir, "FETCH_SIZE"))
        passes["pmc_write"] = rows(os.path.join(out_dir, "WRITE_SIZE"))
    res = {}
    for k in kernels:
        e = {}
        f = per_dispatch(passes["pmc_fetch"], k).get("FETCH_SIZE")
        w = per_dispatch(passes["pmc_write"], k).get("WRITE_SIZE")
        pat = PATTERN.get(k, "stream")
        e["read_pattern"] = pat
        if f:
            raw = f[0] * 1024  # KB -> B
            e["dispatches"] = f[1]
            e["fetch_size_raw_bytes"] = raw
            e["hbm_read_bytes"] = 2 * raw if pat in ("stream", "mixed") else raw
            if pat == "mixed":
                e["hbm_read_bounds"] = [raw, 2 * raw]
        rq = per_dispatch(passes["pmc_rdreq"], k)
        if rq:
            sized = sum(rq.get(c, (0.0, 0))[0] * b for c, b in
                        (("TCC_EA0_RDREQ_32B_sum", 32), ("TCC_EA0_RDREQ_64B_sum", 64), ("TCC_EA0_RDREQ_128B_sum", 128)))
            e["read_requests"] = {c: rq[c][0] for c in rq}
            e["read_bytes_by_request_size"] = sized
            if sized > 0:
                e["hbm_read_bytes"] = sized
                e["hbm_read_source"] = "TCC_EA0_RDREQ by request size"
        if w:
            e["write_size_raw_bytes"] = w[0] * 1024
        if e.get("hbm_read_bytes") is not None and w:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes"] + e["write_size_raw_bytes"]
        e["calibration"] = {k2: v.get("fetch_over_known", v.get("write_over_known")) for k2, v in calib.items()}
        sq = per_dispatch(passes["pmc_sq"], k)
        if sq:
            v = {c: x[0] for c, x in sq.items()}
            e["sq"] = v
            if v.get("SQ_WAVE_CYCLES"):
                e["wait_any_frac"] = v.get("SQ_WAIT_ANY", 0) / v["SQ_WAVE_CYCLES"]
                e["active_inst_frac"] = v.get("SQ_ACTIVE_INST_ANY", 0) / v["SQ_WAVE_CYCLES"]
        tcc = per_dispatch(passes["pmc_tcc"], k)
        if tcc:
            v = {c: x[0] for c, x in tcc.items()}
            e["tcc"] = v
            h, m = v.get("TCC_HIT_sum"), v.get("TCC_MISS_sum")
            if h is not None and m is not None and h + m > 0:
                e["l2_hit_rate"] = h / (h + m)
        res[k] = e
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 96
    # the library the counters were taken from: bench.py uses `traffic` only while this hash matches
    lib = os.environ.get("DOFS_LIB") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "denseopticalflowsegmentation3d_amd", "_build", "libdofs_hip.so")
    import hashlib
    sha = hashlib.sha256(open(lib, "rb").read()).hexdigest()
    print(json.dumps({"batch": batch, "height": 1080, "width": 1920, "lib_sha256": sha, "kernels": res}, indent=1))


if __name__ == "__main__":
    main()
