# heavy-path length threshold of the wave-per-path replay (DOFS_LONG_PATH) vs throughput
set -u
mkdir -p gpurun_out
for i in 1 2; do
for L in ${LENS:-256 128 512 64}; do
  DOFS_LONG_PATH=$L timeout -k 10 300 python bench.py --cpu-frames 0 --no-stages > gpurun_out/lp_$L.log 2>&1 || exit 1
  echo "long_path=$L $(grep -o '"value": [0-9.]*' gpurun_out/lp_$L.log)"
done; done
