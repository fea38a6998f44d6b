# full-size parity with continuations on (three runs: the race it guards is timing dependent)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for C in 1 1 1; do
  DOFS_LONG_CONT=$C timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider -k full_size > gpurun_out/cpar_$C.log 2>&1; rc=$?
  echo "cont=$C rc=$rc"; tail -1 gpurun_out/cpar_$C.log
done
