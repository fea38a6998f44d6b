# Round 6 check 3: the batch sort's onesweep block shape (exp/B rocPRIM's default, exp/C 256 x 12, exp/D 512 x 12):
# parity of C and D on the bench configuration, then a same-box A/B of B, C, D.
set -u
export TMPDIR=/tmp
O=gpurun_out/m3; mkdir -p $O
for v in C D; do
  DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
VARIANTS="B C D" N=2 bash tools/ab.sh || exit 1
# random-gather request sizes by load flavour (tools/gather_micro.hip)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/gm tools/gather_micro.hip || exit 1
timeout -k 10 120 /tmp/gm > $O/gather.txt 2>&1 || { cat $O/gather.txt; exit 1; }
cat $O/gather.txt
timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $O/gpmc -o run --output-format csv -- /tmp/gm > $O/gather_pmc.log 2>&1 || { tail -5 $O/gather_pmc.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/m3/gpmc/**/*counter_collection.csv", recursive=True)[0]
agg = {}
for r in csv.DictReader(open(f)):
    k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
    agg.setdefault(k, []).append(float(r["Counter_Value"]))
names = sorted({k[0] for k in agg})
for n in names:
    if "init" in n: continue
    print(n, {c.replace("TCC_EA0_RDREQ_", ""): round(sum(v) / len(v) / 1e6, 2) for (m, c), v in agg.items() if m == n}, "M per launch")
PY
