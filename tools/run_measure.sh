# Round measurement: PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs), kernel-trace stats, then the
# bench line (N=1, default config) with the probed kernel's traffic from the PMC summary.
set -u
export TMPDIR=/tmp
O=gpurun_out/measure
rm -rf $O; mkdir -p $O
B=${B:-96}
K=${K:-k_boruvka_min}
STREAM=${STREAM---stream}
BENCH="bench.py --steps 3 --warmup 1 --batch $B --cpu-frames 0 --no-stages"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python $BENCH > $O/pmc_fetch.log 2>&1; rc=$?; echo "pmc fetch rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_fetch.log; exit $rc; fi
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python $BENCH > $O/pmc_write.log 2>&1; rc=$?; echo "pmc write rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $O/pmc_write.log; exit $rc; fi
python tools/pmc_summary.py $K $B $O/pmc_fetch $O/pmc_write $STREAM > $O/pmc_summary.json; echo "summary rc=$?"; cat $O/pmc_summary.json
# the trace pass runs the bench's own schedule (10 steps after 3 warmup batches), so the kernel's
# overlap with the other stream matches the timed run its average is compared with
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python bench.py --batch $B --cpu-frames 0 --no-stages --probe $K > $O/trace.log 2>&1; rc=$?; echo "trace rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi
grep "^{" $O/trace.log > $O/trace_bench.json
timeout -k 10 900 python bench.py --batch $B --probe $K --pmc $O/pmc_summary.json > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $O/bench.log
exit $rc
