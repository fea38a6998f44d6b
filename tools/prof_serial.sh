# per-kernel breakdown with the two pipeline phases serialized (DOFS_SERIAL=1), B=32
set -u
export TMPDIR=/tmp
rm -rf gpurun_out/prof_serial
DOFS_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --batch 32 --cpu-frames 0 --no-stages > gpurun_out/prof_serial.log 2>&1; rc=$?; echo "rc=$rc"; grep '^{' gpurun_out/prof_serial.log | cut -c1-200
exit $rc
