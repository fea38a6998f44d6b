# Pipelined and serial kernel traces of the current library (the trace part of tools/round_evidence.sh)
set -u
export TMPDIR=/tmp
O=gpurun_out/trace
mkdir -p $O
rm -rf $O/rocprof $O/rocprof_serial
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rocprof -o run --output-format csv -- python bench.py --cpu-frames 0 --no-h2d > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || exit 1
head -c 250 $O/bench_under_rocprof.json; echo
python tools/one_period.py $O/rocprof > $O/kernel_trace_pipelined_one_period.csv || exit 1
DOFS_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rocprof_serial -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-h2d --no-stages > $O/bench_serial.json 2> $O/bench_serial.err || exit 1
python tools/one_period.py $O/rocprof_serial > $O/kernel_trace_serial_one_batch.csv || exit 1
rm -rf $O/rocprof $O/rocprof_serial
