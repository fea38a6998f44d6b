# Borůvka edge-list contraction: parity (default), then the MST stage time per switch round, then a
# serialized kernel trace at the default switch round
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for L in 0 3 6; do
  DOFS_BLIST=$L timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch 32 --cpu-frames 0 > gpurun_out/blist_$L.log 2>&1; rc=$?
  echo "blist=$L rc=$rc $(grep -o '"value": [0-9.]*\|"mst": [0-9.]*' gpurun_out/blist_$L.log | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
bash tools/prof_serial.sh
