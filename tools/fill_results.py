"""Rewrite DESIGN.md §8 from tools/results_template.md, its RESULT_* fields filled from an evidence directory
(tools/round_evidence.sh → profiles/rNN): python tools/fill_results.py profiles/r06 [DESIGN.md]. Prints the values."""
import csv
import json
import os
import sys

src = sys.argv[1]
path = sys.argv[2] if len(sys.argv) > 2 else "DESIGN.md"


def jl(name):
    t = open(os.path.join(src, name)).read()
    return json.loads(t[t.index("{"):t.rindex("}") + 1])


b = jl("bench_default.json")
m = jl("intraframe_model.json")
r = b["roofline"]
st = b["stages_ms_per_batch"]
cpu = b["cpu_baseline"]
sec = "; ".join(f"`{x['kernel']}` {x['ms_per_batch']} ms, {x.get('frac')} of HBM, traffic {x.get('traffic_over_alg')}× its "
                f"model" for x in r["secondary"][:4])
rows = list(csv.DictReader(open(os.path.join(src, "kernel_trace_pipelined_one_period.csv"))))
end = max(float(x["end_us"]) for x in rows) / 1e3
krt = sum(float(x["dur_us"]) for x in rows if "k_krt_fused" in x["kernel"]) / 1e3
period = (f"a {end:.1f}-ms period: `k_krt_fused` {krt:.1f} ms with every CU (nothing of the other stage runs beside "
          f"it), then this batch's stage B beside the next batch's blur, Borůvka and sort (per-kernel rows in the csv).")
vals = {
    "RESULT_SHA": json.load(open(os.path.join(src, "pmc_kernels.json"))).get("lib_sha256", "?")[:12],
    "RESULT_VALUE": f"{b['value']:,.1f}",
    "RESULT_STEP": f"{b['ms_per_step']}",
    "RESULT_MEDIAN": f"{b['ms_per_step_median']}",
    "RESULT_STAGES": ", ".join(f"{k} {v}" for k, v in st.items()) + " ms",
    "RESULT_CPU": f"{cpu['O2']['value']} Mpixels/s at -O2, {cpu['O0']['value']} at -O0",
    "RESULT_KRT": (f"{r['ms_per_batch']} ms per batch ({r['avg_launch_us'] / 1e3:.1f} ms per launch), "
                   f"{r['achieved']:.0f} GB/s of its 47-B-per-merge model = {r['frac']:.4f} of 8 TB/s, measured traffic "
                   f"{r.get('traffic', 0) / 1e9:.1f} GB per launch = {r.get('traffic_over_alg')}× the model"),
    "RESULT_PATH": f"{r['path_input_roofline_frac']}",
    "RESULT_SEC": sec,
    "RESULT_PERIOD": period,
    "RESULT_4K": f"{m['one_gpu_ms_per_frame']}",
    "RESULT_SPLIT": f"{m.get('projected_speedup_split', m.get('projected_speedup'))}",
    "RESULT_K20": (f"{jl('bench_steps20.json')['value']:,.1f}" if os.path.exists(os.path.join(src, "bench_steps20.json"))
                   else "(not measured)"),
}
sec8 = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "results_template.md")).read()
for k in sorted(vals, key=len, reverse=True):  # (RESULT_SPLIT before RESULT_S...: longest names first)
    sec8 = sec8.replace(k, vals[k])
s = open(path).read()
a, z = s.index("## 8. Results"), s.index("## 9. History")
open(path, "w").write(s[:a] + sec8 + s[z:])
print(json.dumps(vals, indent=1))
