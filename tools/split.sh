set -u
mkdir -p gpurun_out
for S in 0 1; do
 for B in 32 64; do
  DOFS_SPLIT=$S timeout -k 10 600 python bench.py --steps 8 --warmup 2 --batch $B --cpu-frames 0 --no-stages > gpurun_out/split${S}_${B}.log 2>&1; rc=$?; echo "split=$S B=$B rc=$rc $(grep -o '"value": [0-9.]*' gpurun_out/split${S}_${B}.log)"
  if [ $rc -ne 0 ]; then exit $rc; fi
 done
done
