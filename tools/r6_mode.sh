# Run-to-run "modes" of the bench (same library): back-to-back processes, then with pauses between them;
# free device memory printed before each run (is the last process's memory still being released?)
set -u
mkdir -p gpurun_out/mode
lib=${LIB:-denseopticalflowsegmentation3d_amd/_build/libdofs_hip.so}
one() {
  python -c "import torch; f,t=torch.cuda.mem_get_info(); print('free GiB %.1f of %.1f' % (f/2**30, t/2**30))"
  DOFS_LIB=$PWD/$lib timeout -k 10 300 python bench.py --cpu-frames 0 --no-h2d > gpurun_out/mode/$1.log 2>&1 || exit 1
  tail -1 gpurun_out/mode/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_batch']; print('$1', d['value'], d['ms_per_step_median'], 'krt', s['krt'], 'pre', s['preorder'], 'labels', s['labels'])"
}
for i in 1 2 3 4; do one b$i; done
for i in 1 2 3; do sleep ${PAUSE:-40}; one p$i; done
