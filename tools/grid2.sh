set -u
for G in 256 32; do
 for C in 16384 4096 2048; do
  DOFS_LONG_GRID=$G DOFS_GRID_CAP=$C timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch 96 --cpu-frames 0 --no-stages > gpurun_out/g_${G}_$C.log 2>&1; rc=$?; echo "longgrid=$G cap=$C rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/g_${G}_$C.log)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/g_${G}_$C.log; exit $rc; fi
 done
done
