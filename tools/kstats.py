"""Summarise a rocprofv3 kernel_stats.csv (top kernels by total time)."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
for r in rows[:n]:
    m = re.search(r"^(?:void )?(?:dofs::)?([\w:]+?)[<(]", r["Name"]) or re.search(r"(\w+)", r["Name"])
    nm = m.group(1).split("::")[-1]
    if nm == "k_generic":
        m2 = re.search(r"k_generic<dofs::(\w+)>", r["Name"])
        nm = m2.group(1) if m2 else nm
    print(f"{nm[:34]:34s} calls={r['Calls']:>6} total={float(r['TotalDurationNs'])/1e6:9.2f}ms "
          f"avg={float(r['AverageNs'])/1e3:9.1f}us max={float(r['MaxNs'])/1e3:9.1f}us {100*float(r['TotalDurationNs'])/tot:5.1f}%")
