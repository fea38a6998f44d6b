# Run-to-run "modes": is the bench's slow mode tied to the parity of GPU processes on the box?
# Sequence: bench, tiny, tiny, bench, tiny, tiny, bench, bench (tiny = a process that only queries memory)
set -u
mkdir -p gpurun_out/mode
lib=${LIB:-denseopticalflowsegmentation3d_amd/_build/libdofs_hip.so}
tiny() { python -c "import torch; f,t=torch.cuda.mem_get_info(); print('tiny: free GiB %.1f' % (f/2**30))"; }
one() {
  DOFS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --cpu-frames 0 --no-h2d > gpurun_out/mode/$1.log 2>&1 || exit 1
  tail -1 gpurun_out/mode/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_batch']; print('$1', d['value'], d['ms_per_step_median'], 'krt', s['krt'], 'pre', s['preorder'], 'labels', s['labels'])"
}
one c1; tiny; tiny; one c2; tiny; tiny; one c3; one c4
