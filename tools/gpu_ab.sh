# Parity subset on the working build, then a same-box A/B (tools/ab.sh) and a FETCH_SIZE / WRITE_SIZE pass
# of the working build for one kernel. Stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_batch.py} -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ab_pytest.log; if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/ab.sh || exit 1
if [ -n "${PMCK:-}" ]; then
  O=gpurun_out/abpmc; rm -rf $O; mkdir -p $O
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c -d $O/$c -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --cpu-frames 0 --no-stages --no-h2d > $O/$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
  done
  python tools/pmc_kernels.py $O gpurun_out/pmc/fetch_calib.json $PMCK 2>/dev/null > $O/summary.json || true
fi
