# Round-4 measurement at the working tree's library (one call): GPU suite + smoke, rocprofv3 kernel stats
# of the bench, the PMC passes (B = 112, incl. the sized read requests) and the default bench line reading
# that PMC summary (tools/_final4b.sh: config 5's model, the replay / KRT anatomy). Stops at the first
# failing step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n 3 "gpurun_out/$name.log" | cut -c1-300
    [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
rm -rf gpurun_out/prof
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-frames 0 --no-h2d
B=112 bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1; rc=$?; tail -3 gpurun_out/pmc_round.log; [ $rc -eq 0 ] || exit $rc
step bench_final 600 python bench.py --pmc gpurun_out/pmc/pmc_kernels.json
exit 0
