# continuation on/off: parity (on), then bench B=64 with the replay kernels probed.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp


for C in 1 0; do
 for K in k_replay_long KReplay; do
  DOFS_LONG_CONT=$C timeout -k 10 600 python bench.py --steps 6 --warmup 2 --batch 64 --cpu-frames 0 --probe $K > gpurun_out/cont_${C}_$K.log 2>&1; rc=$?
  echo "cont=$C $K rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_batch": [0-9.]*\|"replay": [0-9.]*' gpurun_out/cont_${C}_$K.log | tr "\n" " "; echo
  if [ $rc -ne 0 ]; then exit $rc; fi
 done
done
