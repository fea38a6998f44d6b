cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m3
for v in E B; do
  timeout -k 10 300 python -u tools/stress_determinism.py 20 $PWD/exp/$v/libdofs_hip.so > gpurun_out/m3/stress_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/m3/stress_$v.log)"
done
mkdir -p gpurun_out/m1; sed -n "/^for m in/,\$p" tools/_m1.sh > /tmp/m1loop.sh
export TMPDIR=/tmp
bash /tmp/m1loop.sh
