"""Per-kernel sums of a rocprofv3 --pmc counter_collection.csv (one pass)."""
import collections
import csv
import glob
import re
import sys

f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    m = re.search(r"k_generic<dofs::(\w+)", n) or re.search(r"^(?:void )?(?:dofs::)?([\w:]+?)[<(]", n)
    k = m.group(1).split("::")[-1] if m else n[:24]
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
names = sorted({c for v in acc.values() for c in v})
print("kernel".ljust(22) + "".join(c[3:][:14].rjust(15) for c in names))
for k, v in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:25]:
    print(k[:22].ljust(22) + "".join(f"{v.get(c, 0):15.4g}" for c in names))
