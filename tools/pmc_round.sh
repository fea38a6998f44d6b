# Round measurement of the dominant kernels: FETCH/WRITE calibration (tools/fetch_calib), then separate
# rocprofv3 --pmc passes over a short bench (FETCH_SIZE; WRITE_SIZE; SQ issue/wait; L2 hit/miss), then
# the per-kernel summary (tools/pmc_kernels.py). Every GPU step has its own time limit; the script
# stops at the first failure.
set -u
export TMPDIR=/tmp
O=gpurun_out/pmc
rm -rf $O; mkdir -p $O
B=${B:-96}
KS=${KS:-k_boruvka_min4,k_krt_fused,k_replay_flow,k_pre_sweep,KPathInit,KLift,KFilter,k_blur_fused}
RDREQ="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
BENCH="bench.py --steps 2 --warmup 1 --batch $B --cpu-frames 0 --no-stages --no-h2d"
run() {  # name cmd...
    local name=$1; shift
    timeout -k 10 -s KILL 300 "$@" > $O/$name.log 2>&1; local rc=$?
    echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/$name.log; exit $rc; fi
}
run calib_fetch rocprofv3 --pmc FETCH_SIZE -d $O/calib_fetch -o run --output-format csv -- ./tools/fetch_calib
run calib_write rocprofv3 --pmc WRITE_SIZE -d $O/calib_write -o run --output-format csv -- ./tools/fetch_calib
run calib_rdreq rocprofv3 --pmc $RDREQ -d $O/calib_rdreq -o run --output-format csv -- ./tools/fetch_calib
python tools/calib.py $O/calib_fetch $O/calib_write $O/calib_rdreq > $O/fetch_calib.json || exit 1
cat $O/fetch_calib.json
run pmc_fetch rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python $BENCH
run pmc_write rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python $BENCH
run pmc_sq rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS -d $O/pmc_sq -o run --output-format csv -- python $BENCH
run pmc_rdreq rocprofv3 --pmc $RDREQ -d $O/pmc_rdreq -o run --output-format csv -- python $BENCH
run pmc_tcc rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $O/pmc_tcc -o run --output-format csv -- python $BENCH
python tools/pmc_kernels.py $O $O/fetch_calib.json $KS $B > $O/pmc_kernels.json || exit 1
cat $O/pmc_kernels.json
