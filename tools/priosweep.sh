set -u
for V in 0 1; do
 for B in 64 96; do
  DOFS_PRIO=$V timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch $B --cpu-frames 0 --no-stages > gpurun_out/prio${V}_$B.log 2>&1; rc=$?; echo "prio=$V B=$B rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/prio${V}_$B.log)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/prio${V}_$B.log; exit $rc; fi
 done
done
