# Exact zero weights alone at key 0, passed by the sort fix-up (KZ):
# the whole GPU suite on the variant, the Borůvka kernels' serial durations, then an A/B with two copies of HEAD
set -u
export TMPDIR=/tmp
v=${V:-KZ}
DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/suite_$v.log 2>&1 || { echo "suite $v failed"; tail -30 gpurun_out/suite_$v.log; exit 1; }
tail -1 gpurun_out/suite_$v.log
for x in HB $v; do
  rm -rf gpurun_out/st_$x
  DOFS_LIB=$PWD/exp/$x/libdofs_hip.so DOFS_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/st_$x -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-h2d --no-stages > /dev/null 2>&1 || exit 1
  python - "$x" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/st_{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if any(k in n for k in ("sortfix", "KMstEmit", "trampoline")):
        print(sys.argv[1], n[:60], r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
  rm -rf gpurun_out/st_$x
done
VARIANTS="HB $v HB2" N=${N:-3} bash tools/ab.sh
