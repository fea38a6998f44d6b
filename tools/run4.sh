set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
for B in 4 16; do
  timeout -k 10 600 python bench.py --steps 5 --warmup 2 --batch $B --cpu-frames 0 > gpurun_out/bench_b$B.log 2>&1; rc=$?; echo "bench B=$B rc=$rc"; tail -2 gpurun_out/bench_b$B.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --batch 8 --cpu-frames 0 --no-stages > gpurun_out/rocprof.log 2>&1; echo "rocprof rc=$?"
