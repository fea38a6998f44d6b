# Round 6 check 6: the KRT sweep with pipelined finds (exp/P1 = the working tree) — parity of the KRT paths, then a
# same-box A/B against exp/F (HEAD before it).
set -u
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_config.py tests/test_gpu_batch.py tests/test_gpu_determinism.py tests/test_gpu_lean.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/m6_pytest.log 2>&1 || { tail -30 gpurun_out/m6_pytest.log; exit 1; }
tail -1 gpurun_out/m6_pytest.log
VARIANTS="F P1" N=2 bash tools/ab.sh || exit 1
