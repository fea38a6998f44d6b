"""FETCH_SIZE / WRITE_SIZE calibration on gfx950 (tools/fetch_calib.hip): counter bytes / known bytes.

usage: python tools/calib.py FETCH_DIR WRITE_DIR [RDREQ_DIR] > profiles/<round>/fetch_calib.json

RDREQ_DIR (optional): a pass of TCC_EA0_RDREQ_sum, TCC_EA0_RDREQ_32B_sum, TCC_EA0_RDREQ_64B_sum and
TCC_EA0_RDREQ_128B_sum; the read bytes by request size, 32 R32 + 64 R64 + 128 R128, are compared with
the known bytes as well ("sized_over_known"), the check that this measure needs no per-pattern factor.
"""
import csv
import glob
import json
import os
import sys

GB = 1 << 30
RAND = 1 << 24
KNOWN = {  # kernel-name fragment -> (read bytes, written bytes) per launch
    "rd<int>": (GB, 0), "rd<unsigned long>": (GB, 0), "rd<HIP_vector_type<int, 4u> >": (GB, 0),
    "wr<int>": (0, GB), "wr<unsigned long>": (0, GB), "wr<HIP_vector_type<int, 4u> >": (0, GB),
    "gather<HIP_vector_type<int, 4u> >": (16 * RAND, 0), "gather<int>": (4 * RAND, 0),
    "scatter8": (0, 8 * RAND),
}
LABEL = {"rd<int>": "read 4 B/lane", "rd<unsigned long>": "read 8 B/lane",
         "rd<HIP_vector_type<int, 4u> >": "read 16 B/lane", "wr<int>": "write 4 B/lane",
         "wr<unsigned long>": "write 8 B/lane", "wr<HIP_vector_type<int, 4u> >": "write 16 B/lane",
         "gather<HIP_vector_type<int, 4u> >": "random 16-B reads", "gather<int>": "random 4-B reads",
         "scatter8": "random 8-B writes"}


SIZED = {"TCC_EA0_RDREQ_32B_sum": 32, "TCC_EA0_RDREQ_64B_sum": 64, "TCC_EA0_RDREQ_128B_sum": 128}


def per_kernel(d, counter, scale=1024):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            name = r["Kernel_Name"]
            for k in KNOWN:
                if name.startswith(("void " + k + "(", k + "(")):
                    out.setdefault(k, {}).setdefault(r["Dispatch_Id"], 0.0)
                    out[k][r["Dispatch_Id"]] += float(r["Counter_Value"]) * scale  # KB -> B
    return {k: sum(v.values()) / len(v) for k, v in out.items()}


def main():
    fetch = per_kernel(sys.argv[1], "FETCH_SIZE")
    write = per_kernel(sys.argv[2], "WRITE_SIZE")
    sized, reqs = {}, {}
    if len(sys.argv) > 3:
        for c, b in SIZED.items():
            for k, v in per_kernel(sys.argv[3], c, scale=b).items():
                sized[k] = sized.get(k, 0.0) + v
        reqs = per_kernel(sys.argv[3], "TCC_EA0_RDREQ_sum", scale=1)
    res = {}
    for k, (rb, wb) in KNOWN.items():
        e = {"known_read_bytes": rb, "known_write_bytes": wb,
             "fetch_size_bytes": fetch.get(k), "write_size_bytes": write.get(k)}
        if rb and fetch.get(k) is not None:
            e["fetch_over_known"] = round(fetch[k] / rb, 4)
        if wb and write.get(k) is not None:
            e["write_over_known"] = round(write[k] / wb, 4)
        if rb and k in sized:
            e["sized_read_bytes"] = sized[k]
            e["sized_over_known"] = round(sized[k] / rb, 4)
            e["read_requests"] = reqs.get(k)
        res[LABEL[k]] = e
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
