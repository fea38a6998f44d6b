# Kernel-time anatomy of the bench workload (1080p, B = 112): a serial run (DOFS_SERIAL=1: the phases back
# to back, so each kernel's duration is its own work) and the pipelined run (kernel trace for
# tools/timeline.py: per-stream busy time and overlap). Each step has its own time limit.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_serial gpurun_out/prof_pipe
ARGS="--steps 3 --warmup 1 --cpu-frames 0 --no-stages --no-h2d"
DOFS_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run --output-format csv -- python bench.py $ARGS > gpurun_out/prof_serial.log 2>&1 || { echo "serial rc=$?"; tail -5 gpurun_out/prof_serial.log; exit 1; }
echo "== serial"; tail -1 gpurun_out/prof_serial.log | cut -c1-300
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pipe -o run --output-format csv -- python bench.py $ARGS > gpurun_out/prof_pipe.log 2>&1 || { echo "pipe rc=$?"; tail -5 gpurun_out/prof_pipe.log; exit 1; }
echo "== pipelined"; tail -1 gpurun_out/prof_pipe.log | cut -c1-300
for d in prof_serial prof_pipe; do
  f=$(find gpurun_out/$d -name "*kernel_stats.csv" | head -1); echo "== $d top kernels"; python tools/kstats.py $f 30
done
python tools/timeline.py gpurun_out/prof_pipe 2.0 || true
