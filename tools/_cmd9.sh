# GPU check of the working tree: full -m gpu suite, smoke, default bench, one 4K frame (config 5 model)
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?; tail -2 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 || exit $?; tail -1 gpurun_out/bench.log | cut -c1-300
timeout -k 10 300 python tools/bench_intraframe.py --model 4 > gpurun_out/intraframe_model.log 2>&1 || exit $?; tail -1 gpurun_out/intraframe_model.log
