cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/m10
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/psm tools/partial_store_micro.hip || exit 1
timeout -k 10 60 /tmp/psm || exit 1
rm -rf gpurun_out/m10/f gpurun_out/m10/w
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/m10/f -o run --output-format csv -- /tmp/psm > /dev/null 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/m10/w -o run --output-format csv -- /tmp/psm > /dev/null 2>&1 || exit 1
python3 - <<PY
import csv,glob
for tag in ('f','w'):
    f=glob.glob('gpurun_out/m10/%s/**/*counter_collection.csv'%tag, recursive=True)[0]
    rows=list(csv.DictReader(open(f)))
    agg={}
    for r in rows:
        n=r['Kernel_Name'].split('(')[0]
        agg.setdefault(n,[]).append(float(r['Counter_Value']))
    for n,v in agg.items(): print(tag, n, [round(x/1e6,1) for x in v][:3], 'MB per launch (first 3)')
PY
for v in Q1 Q2; do
  DOFS_LIB=$PWD/exp/$v/libdofs_hip.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_config.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/m10/pytest_$v.log 2>&1 || { tail -15 gpurun_out/m10/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/m10/pytest_$v.log)"
done
VARIANTS="E=E Q1=Q1 Q2=Q2" N=2 bash tools/ab_env.sh
