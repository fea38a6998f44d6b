set -u
mkdir -p gpurun_out
DOFS_LONG_WAVES=1 timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_w1.log 2>&1; rc=$?; echo "pytest(1 wave) rc=$rc"; tail -2 gpurun_out/pytest_w1.log
if [ $rc -ne 0 ]; then exit $rc; fi
for V in 3 1; do
 for B in 64 96; do
  DOFS_LONG_WAVES=$V timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch $B --cpu-frames 0 > gpurun_out/waves${V}_$B.log 2>&1; rc=$?; echo "waves=$V B=$B rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/waves${V}_$B.log) $(grep -o '"replay": [0-9.]*' gpurun_out/waves${V}_$B.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
 done
done
