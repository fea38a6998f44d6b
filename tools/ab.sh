# Same-box A/B(/C...) of builds of the library (exp/A, exp/B, ...: VARIANTS="A B C"; built with `make OUT=...`; exp/ is git-ignored but travels to the box), alternating
# bench runs so box-to-box variance cancels. Prints value and stage times per run.
set -u
N=${N:-3}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in ${VARIANTS:-A B}; do
    # TINY=1: a process that only queries device memory before each run (the box's run-to-run modes, DESIGN.md
    # §9.1: with one between them, every bench run of tools/r6_mode.sh ran in the fast mode)
    if [ -n "${TINY:-}" ]; then python -c "import torch; torch.cuda.mem_get_info()" || exit 1; fi
    DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 300 python bench.py --cpu-frames 0 ${ARGS:-} > gpurun_out/ab_$v$i.log 2>&1 || exit 1
    tail -1 gpurun_out/ab_$v$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_batch'] or {}; print('$v', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), ' '.join(f'{k}={v}' for k, v in s.items()))"
  done
done
