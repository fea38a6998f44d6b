"""Copy one measurement run (tools/run_measure.sh → gpurun_out/measure) into profiles/<name>/.

Keeps the rocprofv3 kernel stats, the probed kernel's per-dispatch PMC rows, the PMC summary, the
bench lines, and a check that the bench's event-timed average launch of the probed kernel agrees
with rocprofv3's average for the same kernel in the same command.
"""
import csv
import json
import os
import shutil
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/measure"
dst = os.path.join("profiles", sys.argv[2] if len(sys.argv) > 2 else "r01")
os.makedirs(dst, exist_ok=True)
summ = json.load(open(os.path.join(src, "pmc_summary.json")))
kernel = summ["kernel"]
shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
shutil.copy(os.path.join(src, "pmc_summary.json"), os.path.join(dst, "pmc_summary.json"))
for name in ("bench.log", "trace.log"):
    lines = [ln for ln in open(os.path.join(src, name)) if ln.startswith("{")]
    open(os.path.join(dst, "bench.json" if name == "bench.log" else "trace_bench.json"), "w").write(lines[-1])
for cnt in ("fetch", "write"):
    rows = [r for r in csv.DictReader(open(os.path.join(src, f"pmc_{cnt}", "run_counter_collection.csv")))
            if f"dofs::{kernel}" in r["Kernel_Name"]]
    with open(os.path.join(dst, f"pmc_{cnt}_{kernel}.csv"), "w", newline="") as f:
        wr = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
        wr.writeheader()
        wr.writerows(rows)
stats = [r for r in csv.DictReader(open(os.path.join(dst, "kernel_stats.csv")))
         if f"dofs::{kernel}>" in r["Name"] or f"dofs::{kernel}(" in r["Name"]]
tb = json.loads(open(os.path.join(dst, "trace_bench.json")).read())
rp_avg = float(stats[0]["AverageNs"]) / 1e3
ev_avg = tb["roofline"]["avg_launch_us"]
msg = (f"{kernel}: rocprofv3 average {rp_avg:.1f} us over {stats[0]['Calls']} calls (whole command incl. warmup);"
       f" bench device-event average {ev_avg:.1f} us over {tb['roofline']['launches']} timed launches;"
       f" ratio {ev_avg / rp_avg:.3f}\n")
open(os.path.join(dst, "probe_vs_rocprof.txt"), "w").write(msg)
print(msg, end="")
