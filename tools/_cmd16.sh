mkdir -p gpurun_out
timeout -k 10 400 python bench.py --frames 512 --cpu-frames 0 --no-h2d > gpurun_out/config4_1gpu.log 2>&1 || exit $?; tail -1 gpurun_out/config4_1gpu.log | cut -c1-300
timeout -k 10 300 python tools/bench_intraframe.py --model 4 > gpurun_out/intraframe_model.log 2>&1 || exit $?; tail -1 gpurun_out/intraframe_model.log
