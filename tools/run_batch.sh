set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 32 64; do
  timeout -k 10 600 python bench.py --steps 3 --warmup 1 --batch $B --cpu-frames 0 > gpurun_out/bench_b$B.log 2>&1; rc=$?; echo "bench B=$B rc=$rc"; tail -1 gpurun_out/bench_b$B.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
