# Round 6 check 2: the stale-sector micro (extended), the replay parity subset, a same-box A/B of the replay
# publish (exp/A: three 8-B stores, exp/B: 16 + 8), and WRITE_SIZE of k_replay_flow on both. Stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/m2; mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/ssm tools/stale_sector_micro.hip || exit 1
timeout -k 10 120 /tmp/ssm 2000 > $O/stale.json 2>&1 || { echo micro failed; exit 1; }
grep -c '"cross_xcd_stale": 0' $O/stale.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_flow_order.py tests/test_gpu_lean.py tests/test_gpu_determinism.py tests/test_gpu_bench_config.py tests/test_gpu_replay_modes.py tests/test_gpu_flow_giveup.py tests/test_gpu_intraframe.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
N=2 bash tools/ab.sh || exit 1
for v in A B; do
  timeout -k 10 -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/w_$v -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --cpu-frames 0 --no-stages --no-h2d > $O/w_$v.log 2>&1 || { echo pmc $v failed; exit 1; }
done
python - <<'PY'
import csv, glob
for v in "AB":
    fs = glob.glob(f"gpurun_out/m2/w_{v}/**/*counter_collection.csv", recursive=True)
    tot = {}
    for f in fs:
        for r in csv.DictReader(open(f)):
            n = r.get("Kernel_Name", "")
            if "k_replay_flow" in n:
                key = "long" if "true" in n else "short"
                tot.setdefault(key, []).append(float(r["Counter_Value"]))
    print(v, {k: (len(x), round(sum(x) / len(x) / 1e9, 3)) for k, x in tot.items()}, "GB per launch (WRITE_SIZE KB units?)")
PY
