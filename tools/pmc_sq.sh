# SQ issue/wait counters per kernel (one PMC pass), B=32, serialized phases
set -u
export TMPDIR=/tmp
O=gpurun_out/pmc_sq
rm -rf $O; mkdir -p $O
DOFS_SERIAL=1 timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $O/p -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --batch 32 --cpu-frames 0 --no-stages > $O/log 2>&1; rc=$?; echo "rc=$rc"
exit $rc
