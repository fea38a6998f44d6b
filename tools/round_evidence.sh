# End-of-round evidence in one gpurun call (each GPU step under its own time limit, stop at the first
# failure): the PMC passes (tools/pmc_round.sh, B = 112), then the bench with that PMC summary, the
# rocprofv3 kernel stats of the same bench and one pipelined period of its trace, the serial kernel trace,
# config 5's model, smoke() and the determinism stress. Outputs under gpurun_out/evidence/.
set -u
export TMPDIR=/tmp
O=gpurun_out/evidence
mkdir -p $O
B=112 KS=k_boruvka_min4,k_boruvka_recs\<false\>,k_krt_fused,k_replay_flow,k_pre_sweep,KPathInit,KLift,KFilter,k_blur_fused bash tools/pmc_round.sh > $O/pmc_round.log 2>&1 || { tail -20 $O/pmc_round.log; exit 1; }
tail -3 $O/pmc_round.log
cp gpurun_out/pmc/pmc_kernels.json gpurun_out/pmc/fetch_calib.json $O/
timeout -k 10 600 python bench.py --pmc $O/pmc_kernels.json > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
head -c 300 $O/bench_default.json; echo
rm -rf $O/rocprof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rocprof -o run --output-format csv -- python bench.py --cpu-frames 0 --no-h2d > $O/bench_under_rocprof.json 2> $O/bench_under_rocprof.err || exit 1
python tools/one_period.py $O/rocprof > $O/kernel_trace_pipelined_one_period.csv || exit 1
timeout -k 10 300 python tools/bench_intraframe.py --model 4 > $O/intraframe_model.json 2>&1 || exit 1
tail -1 $O/intraframe_model.json | cut -c1-300
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
# one B = 112 batch per step with the two stages back to back (DOFS_SERIAL=1): every kernel's duration is
# its own work, not time queued behind the other stage (stage-B kernels in particular)
rm -rf $O/rocprof_serial
DOFS_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rocprof_serial -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-frames 0 --no-h2d --no-stages > $O/bench_serial.json 2> $O/bench_serial.err || exit 1
head -c 300 $O/bench_serial.json; echo
python tools/one_period.py $O/rocprof_serial > $O/kernel_trace_serial_one_batch.csv || exit 1
# determinism under workspace reuse: the fixed-job split repeated, records identical every time
timeout -k 10 600 python tools/stress_determinism.py 40 - 1 > $O/stress_determinism_keep.log 2>&1 || { tail -5 $O/stress_determinism_keep.log; exit 1; }
tail -1 $O/stress_determinism_keep.log
timeout -k 10 600 python tools/stress_determinism.py 40 - 0 > $O/stress_determinism_default.log 2>&1 || { tail -5 $O/stress_determinism_default.log; exit 1; }
tail -1 $O/stress_determinism_default.log
