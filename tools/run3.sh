set -u
mkdir -p gpurun_out
timeout -k 10 120 ./tools/replay_micro > gpurun_out/micro.log 2>&1; echo "micro rc=$?"; cat gpurun_out/micro.log
bash tools/gpu_check.sh
