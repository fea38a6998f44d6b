# Pipeline depth vs batch size on one GPU box: the bench with DOFS_SLOTS (workspaces in flight, 2 or 3)
# and --batch (frames per step) varied together, two interleaved reps. Fewer slots free HBM for larger
# batches (each workspace is ~0.75 GB per 1080p frame).
#   bash tools/slots_sweep.sh
mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
 for cfg in "3 96" "2 96" "2 128" "2 144"; do set -- $cfg
  DOFS_SLOTS=$1 timeout -k 10 300 python bench.py --cpu-frames 0 --no-h2d --batch $2 > gpurun_out/slots_$1_$2_$i.log 2>&1 || { echo "slots=$1 B=$2 failed rc=$?"; tail -3 gpurun_out/slots_$1_$2_$i.log; exit 1; }
  echo "slots=$1 B=$2 $(grep -o '"value": [0-9.]*\|"ms_per_step_median": [0-9.]*' gpurun_out/slots_$1_$2_$i.log | tr '\n' ' ')"
 done
done
