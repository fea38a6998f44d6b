# Round 6 check 7: KRT phase anatomy (tools/krt_timing.py, -DDOFS_KRT_TIMING builds) of HEAD (exp/KF) and the
# pipelined-find sweep (exp/KP), B = 112.
set -u
export TMPDIR=/tmp
for v in KF KP; do
  DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 300 python tools/krt_timing.py 112 3 > gpurun_out/m7_$v.json 2>&1 || { tail -5 gpurun_out/m7_$v.json; exit 1; }
done
python - <<'PY'
import json
for v in ("KF", "KP"):
    t = open(f"gpurun_out/m7_{v}.json").read(); d = json.loads(t[t.index("{"):])
    print(v, {k: x["us_per_block"] for k, x in d["phases"].items()}, d["sweep"])
PY
