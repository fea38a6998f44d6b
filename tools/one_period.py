"""One period of the bench from a rocprofv3 kernel trace: the kernels between the starts of two consecutive
k_krt_fused launches in the middle of the run (inside the timed steps: the bench's stage-timing pass at the end
runs its batches serially), as csv (kernel, stream_id, start_us, end_us, dur_us; times from the period start).
usage: python tools/one_period.py TRACE_DIR > period.csv"""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
starts = sorted(int(r["Start_Timestamp"]) for r in rows if "k_krt_fused" in r["Kernel_Name"])
if len(starts) < 3:
    sys.exit("fewer than three k_krt_fused launches")
m = len(starts) // 2
t0, t1 = starts[m - 1], starts[m]
w = csv.writer(sys.stdout)
w.writerow(["kernel", "stream_id", "start_us", "end_us", "dur_us"])
for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if t0 <= s < t1:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        w.writerow([name[:90], r[key], round((s - t0) / 1e3, 2), round((e - t0) / 1e3, 2), round((e - s) / 1e3, 2)])
