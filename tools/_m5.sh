cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/m5
for v in P F E; do
  timeout -k 10 300 python -u tools/stress_determinism.py 20 $PWD/exp/$v/libdofs_hip.so > gpurun_out/m5/stress_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/m5/stress_$v.log)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
