# workgroups per frame of the long-path replay (DOFS_LONG_GRID) vs throughput
set -u
mkdir -p gpurun_out
for i in 1 2; do
for G in ${GRIDS:-256 128 160 192}; do
  DOFS_LONG_GRID=$G timeout -k 10 300 python bench.py --cpu-frames 0 --no-stages > gpurun_out/lg_$G.log 2>&1 || exit 1
  echo "long_grid=$G $(grep -o '"value": [0-9.]*' gpurun_out/lg_$G.log)"
done; done
