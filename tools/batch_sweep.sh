# frames per batch vs throughput (the replay's latency-bound chain is amortised over more frames)
set -u
mkdir -p gpurun_out
for Bt in ${BATCHES:-96 128 160}; do
  timeout -k 10 400 python bench.py --cpu-frames 0 --no-stages --batch $Bt > gpurun_out/bs_$Bt.log 2>&1 || { tail -3 gpurun_out/bs_$Bt.log; exit 1; }
  echo "batch=$Bt $(grep -o '"value": [0-9.]*' gpurun_out/bs_$Bt.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bs_$Bt.log)"
done
