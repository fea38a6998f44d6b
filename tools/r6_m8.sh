# Round 6 check 8: k_boruvka_min4 from KBoruvkaFirst's edge ranks (working tree, _build and exp/R1) — the whole GPU
# suite on the working build, then a same-box A/B against exp/F (HEAD before it).
set -u
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/m8_pytest.log 2>&1 || { tail -30 gpurun_out/m8_pytest.log; exit 1; }
tail -1 gpurun_out/m8_pytest.log
VARIANTS="F R1" N=3 bash tools/ab.sh || exit 1
