"""Summarise rocprofv3 --pmc passes for one kernel into the JSON bench.py reads as roofline.traffic.

usage: python tools/pmc_summary.py KERNEL BATCH FETCH_DIR WRITE_DIR [--stream] > summary.json

FETCH_DIR / WRITE_DIR: rocprofv3 -d outputs of separate passes (--pmc FETCH_SIZE, --pmc WRITE_SIZE;
one counter per pass: MI355X_MICROARCH.md §rocprofv3 PMC slots). Per-dispatch values of the kernel are
averaged. Correction (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports exactly half the bytes of
a wide coalesced streaming read (128-B requests tallied at 64 B); --stream doubles it for kernels whose
reads are coalesced rows (k_boruvka_min: label and flow rows of a tile). WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys


def rows(d):
    fs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    out = []
    for f in fs:
        out.extend(csv.DictReader(open(f)))
    return out


def per_dispatch(d, kernel, counter):
    vals = {}
    for r in rows(d):
        name = r.get("Kernel_Name", "")
        if not (f"dofs::{kernel}>" in name or f"dofs::{kernel}(" in name) or r.get("Counter_Name") != counter:
            continue
        vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    kernel, batch, fdir, wdir = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    stream = "--stream" in sys.argv[5:]
    f = per_dispatch(fdir, kernel, "FETCH_SIZE")
    w = per_dispatch(wdir, kernel, "WRITE_SIZE")
    # rocprofv3 reports FETCH_SIZE / WRITE_SIZE in KB
    fetch = sum(f) / len(f) * 1024 * (2 if stream else 1) if f else None
    write = sum(w) / len(w) * 1024 if w else None
    out = {"kernel": kernel, "batch": batch, "dispatches": [len(f), len(w)],
           "fetch_size_bytes_per_launch": fetch, "write_size_bytes_per_launch": write,
           "hbm_bytes_per_launch": (fetch + write) if fetch is not None and write is not None else None,
           "fetch_correction": "x2 (gfx950 streaming-read tally)" if stream else "none",
           "note": "FETCH_SIZE + WRITE_SIZE per launch (memory-side requests; Infinity-Cache hits counted)"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
