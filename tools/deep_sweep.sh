set -u
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
for V in 2048 1024 512; do
  L=denseopticalflowsegmentation3d_amd/_build/libdofs_hip.so
  if [ $V != 2048 ]; then L=denseopticalflowsegmentation3d_amd/_build/libdofs_hip_deep$V.so; fi
  DOFS_LIB=$L DOFS_DEEP_S=$V timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch 32 --cpu-frames 0 > gpurun_out/bench_deep$V.log 2>&1; rc=$?; echo "deep=$V rc=$rc"; tail -1 gpurun_out/bench_deep$V.log | cut -c1-100
  grep -o '"stages_ms_per_batch.*' gpurun_out/bench_deep$V.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
