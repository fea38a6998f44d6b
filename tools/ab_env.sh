# Same-box comparison of (library, environment) variants, alternating bench runs so box-to-box variance
# cancels. VARIANTS="name=libdir[,VAR=value...] ..." (libdir under exp/), e.g.
#   VARIANTS="A=A B=B B256=B,DOFS_FLOW_LONG=256 B128=B,@--batch=128" N=2 bash tools/ab_env.sh  (@: a bench argument)
set -u
N=${N:-2}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for spec in $VARIANTS; do
    name=${spec%%=*}
    rest=${spec#*=}
    lib=${rest%%,*}
    envs=""
    bargs=""
    if [ "$rest" != "$lib" ]; then
      for tok in $(echo "${rest#*,}" | tr ',' ' '); do
        case $tok in @*) bargs="$bargs ${tok#@}" ;; *) envs="$envs $tok" ;; esac
      done
    fi
    if [ -n "${TINY:-}" ]; then python -c "import torch; torch.cuda.mem_get_info()" || exit 1; fi  # (tools/ab.sh)
    env $envs DOFS_LIB=$PWD/exp/$lib/libdofs_hip.so timeout -k 10 300 python bench.py --cpu-frames 0 --no-h2d ${ARGS:-} $bargs > gpurun_out/abe_$name$i.log 2>&1 || exit 1
    tail -1 gpurun_out/abe_$name$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_batch'] or {}; print('$name', d['value'], d['ms_per_step'], d.get('ms_per_step_median'), ' '.join(f'{k}={v}' for k, v in s.items()))"
  done
done
