set -u
mkdir -p gpurun_out
for B in 48 64 96 128; do
  timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch $B --cpu-frames 0 --no-stages > gpurun_out/bs_$B.log 2>&1; rc=$?; echo "B=$B rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/bs_$B.log)"
  if [ $rc -ne 0 ]; then tail -3 gpurun_out/bs_$B.log; exit $rc; fi
done
