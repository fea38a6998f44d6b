# Round measurement at the working tree's library: GPU suite + smoke + rocprofv3 kernel stats of the
# bench, the PMC passes (B = 112), then the default bench line reading that PMC summary.
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
step pytest_gpu 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step rocprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --cpu-frames 0 --no-h2d
B=112 bash tools/pmc_round.sh > gpurun_out/pmc_round.log 2>&1; rc=$?; tail -3 gpurun_out/pmc_round.log; [ $rc -eq 0 ] || exit $rc
step bench_final 500 python bench.py --pmc gpurun_out/pmc/pmc_kernels.json
step intraframe_model 300 python tools/bench_intraframe.py --model 4
