# KRT stage anatomy: the sweep (k_krt_seq, one workgroup per frame) and the LDS blocks (k_dnc_deep) as
# separate serial launches (DOFS_FUSED=0 DOFS_SERIAL=1), at two batch sizes, next to the fused kernel.
set -u
mkdir -p gpurun_out/krt
run() {  # name env... -- args
    local name=$1; shift
    timeout -k 10 300 env "$@" > gpurun_out/krt/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/krt/$name.log; exit 1; }
    tail -1 gpurun_out/krt/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', d['value'], [(k['kernel'], k['ms_per_batch'], k['launches'], k['avg_launch_us']) for k in r['top_kernels_by_time']], d.get('stages_ms_per_batch'))"
}
B="python bench.py --cpu-frames 0 --no-h2d --steps 3 --warmup 1"
run unfused96 DOFS_FUSED=0 DOFS_SERIAL=1 $B --batch 96 --probe k_boruvka_min,k_krt_seq,k_dnc_deep
run unfused16 DOFS_FUSED=0 DOFS_SERIAL=1 $B --batch 16 --probe k_boruvka_min,k_krt_seq,k_dnc_deep
run unfused4 DOFS_FUSED=0 DOFS_SERIAL=1 $B --batch 4 --probe k_boruvka_min,k_krt_seq,k_dnc_deep
run fused96 DOFS_SERIAL=1 $B --batch 96 --probe k_boruvka_min,k_krt_fused
run fused96all DOFS_FUSED_EXTRA=256 DOFS_SERIAL=1 $B --batch 96 --probe k_boruvka_min,k_krt_fused
