# Round-4 measurement at the working tree's library (one call): GPU suite + smoke, rocprofv3 kernel stats
# of the bench, the PMC passes (B = 112, incl. the sized read requests), the default bench line reading
# that PMC summary, config 5's model, and the replay / KRT anatomy. Stops at the first failing step.
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
step intraframe_model 300 python tools/bench_intraframe.py --model 4
P=denseopticalflowsegmentation3d_amd/_build/prof/libdofs_hip.so
step flow1080 300 env DOFS_SERIAL=1 python tools/flow_stats.py 112 2
step flow4k 300 env DOFS_SERIAL=1 H=2160 W=3840 python tools/flow_stats.py 1 3
step flow1080_prof 300 env DOFS_SERIAL=1 DOFS_LIB=$P python tools/flow_stats.py 112 2
step flow4k_prof 300 env DOFS_SERIAL=1 DOFS_LIB=$P H=2160 W=3840 python tools/flow_stats.py 1 3
step krt_timing 300 env DOFS_LIB=denseopticalflowsegmentation3d_amd/_build/krt/libdofs_hip.so python tools/krt_timing.py 112 2
exit 0
