# k_krt_fused workgroups (B + DOFS_FUSED_EXTRA, capped at the CU count) vs end-to-end throughput
set -u
mkdir -p gpurun_out
for E in ${EXTRAS:-160 128 96 64 160 128 96 64}; do
  DOFS_FUSED_EXTRA=$E timeout -k 10 300 python bench.py --cpu-frames 0 --no-stages > gpurun_out/ex_$E.log 2>&1 || exit 1
  echo "extra=$E $(grep -o '"value": [0-9.]*' gpurun_out/ex_$E.log)"
done
