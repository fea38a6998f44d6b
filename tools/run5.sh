# GPU session: parity tests, then the pipelined bench at B=32 and B=64.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for B in 32 64; do
  timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch $B --cpu-frames 0 > gpurun_out/bench_b$B.log 2>&1; rc=$?; echo "bench B=$B rc=$rc"; tail -2 gpurun_out/bench_b$B.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
