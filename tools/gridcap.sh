# grid-cap sweep: parity first, then the B=32 bench per cap value
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for C in 4096 16384 0; do
  DOFS_GRID_CAP=$C timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch 32 --cpu-frames 0 > gpurun_out/bench_cap$C.log 2>&1; rc=$?; echo "cap=$C rc=$rc"; tail -1 gpurun_out/bench_cap$C.log | cut -c1-120
  grep -o '"stages_ms_per_batch.*' gpurun_out/bench_cap$C.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
