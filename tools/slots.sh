set -u
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for S in 2 3; do
 for B in 64 96; do
  DOFS_SLOTS=$S timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch $B --cpu-frames 0 --no-stages > gpurun_out/slots${S}_$B.log 2>&1; rc=$?; echo "slots=$S B=$B rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/slots${S}_$B.log)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/slots${S}_$B.log; exit $rc; fi
 done
done
