# Same-box comparison of _ab/A against _ab/B under several environment settings (VARIANTS="ENV=1 ENV=2 ...").
set -u
N=${N:-2}
mkdir -p gpurun_out
for i in $(seq 1 $N); do
  for v in A ${VARIANTS:-B}; do
    lib=A; envs=""
    if [ "$v" != A ]; then lib=B; [ "$v" != B ] && envs="$v"; fi
    env $envs DOFS_LIB=$PWD/_ab/$lib/libdofs_hip.so timeout -k 10 300 python bench.py --cpu-frames 0 --no-h2d ${ARGS:-} > gpurun_out/ab3_$i.log 2>&1 || exit 1
    tail -1 gpurun_out/ab3_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['stages_ms_per_batch']; print('$v', d['value'], d['ms_per_step'], ' '.join(f'{k}={v}' for k, v in s.items()))"
  done
done
