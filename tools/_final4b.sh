# Round-4 measurement, second call (tools/_final4.sh has the suite, the profiles, the PMC passes and the
# bench line): config 5's model and the replay / KRT anatomy at the same library.
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
step intraframe_model 300 python tools/bench_intraframe.py --model 4
P=denseopticalflowsegmentation3d_amd/_build/prof/libdofs_hip.so
step flow1080 300 env DOFS_SERIAL=1 python tools/flow_stats.py 112 2
step flow4k 300 env DOFS_SERIAL=1 H=2160 W=3840 python tools/flow_stats.py 1 3
step flow1080_prof 300 env DOFS_SERIAL=1 DOFS_LIB=$P python tools/flow_stats.py 112 2
step flow4k_prof 300 env DOFS_SERIAL=1 DOFS_LIB=$P H=2160 W=3840 python tools/flow_stats.py 1 3
step krt_timing 300 env DOFS_LIB=denseopticalflowsegmentation3d_amd/_build/krt/libdofs_hip.so python tools/krt_timing.py 112 2
exit 0
