# Per-kernel durations of one B = 112 bench workload twice: with the two pipeline stages serialised on one
# stream (DOFS_SERIAL=1: each kernel alone, its duration is its work) and pipelined (the default: durations
# include the other stage's interference and dispatch waits). rocprofv3 --kernel-trace --stats; each run
# under its own time limit; outputs under gpurun_out/prof_{serial,pipe}/.
set -u
export TMPDIR=/tmp
B=${B:-112}
for mode in serial pipe; do
  rm -rf gpurun_out/prof_$mode
  if [ $mode = serial ]; then export DOFS_SERIAL=1; else unset DOFS_SERIAL; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$mode -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --batch $B --cpu-frames 0 --no-stages --no-h2d > gpurun_out/prof_$mode.log 2>&1
  rc=$?; echo "$mode rc=$rc"; grep '^{' gpurun_out/prof_$mode.log | cut -c1-160
  [ $rc -ne 0 ] && exit $rc
done
exit 0
