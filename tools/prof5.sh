# rocprofv3 kernel stats of the bench at B=32 (per-kernel breakdown).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --batch 32 --cpu-frames 0 --no-stages > gpurun_out/rocprof.log 2>&1; rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/rocprof.log
exit $rc
