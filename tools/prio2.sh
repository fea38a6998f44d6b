set -u
mkdir -p gpurun_out
for i in 1 2; do
for P in 0 2; do for E in 128 160; do
  DOFS_PRIO=$P DOFS_FUSED_EXTRA=$E timeout -k 10 300 python bench.py --cpu-frames 0 --no-stages > gpurun_out/pr_${P}_${E}.log 2>&1 || exit 1
  echo "prio=$P extra=$E $(grep -o '"value": [0-9.]*' gpurun_out/pr_${P}_${E}.log)"
done; done; done
