# GPU session: the GPU suite, smoke, the default bench line, and the replay anatomy (flow_stats) at the
# bench shape (1080p, B = 112) and config 5's shape (one 4K frame). Stops at the first failing step.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -n ${TAILN:-4} "gpurun_out/$name.log" | cut -c1-400
    [ $rc -eq 0 ] || exit $rc
}
if [ -z "${SKIP_TESTS:-}" ]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${TESTS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ -z "${SKIP_BENCH:-}" ]; then
step bench 600 python bench.py ${BENCH_ARGS:-}
fi
if [ -n "${VARIANTS:-}" ]; then  # same-box A/B of library / environment variants (tools/ab_env.sh)
timeout -k 10 900 bash tools/ab_env.sh || exit 1
fi
if [ -n "${ANATOMY:-}" ]; then
P=denseopticalflowsegmentation3d_amd/_build/prof/libdofs_hip.so
step flow1080 300 env DOFS_SERIAL=1 python tools/flow_stats.py 112 2
step flow4k 300 env DOFS_SERIAL=1 H=2160 W=3840 python tools/flow_stats.py 1 3
step flow1080_prof 300 env DOFS_SERIAL=1 DOFS_LIB=$P python tools/flow_stats.py 112 2
step flow4k_prof 300 env DOFS_SERIAL=1 DOFS_LIB=$P H=2160 W=3840 python tools/flow_stats.py 1 3
step flow4k_prof_nopipe 300 env DOFS_FLOW_PIPE=0 DOFS_SERIAL=1 DOFS_LIB=$P H=2160 W=3840 python tools/flow_stats.py 1 3
step intraframe 300 python tools/bench_intraframe.py --model 4
fi
if [ -n "${KRT:-}" ]; then
step krt_timing 300 env DOFS_LIB=denseopticalflowsegmentation3d_amd/_build/krt/libdofs_hip.so python tools/krt_timing.py 112 2
fi
exit 0
