# A/B timing of library variants (CEP_LIB) after the cf parity tests.
# usage: LIBS="libcep.so libcep_b.so" bash scripts/cmp.sh
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/cmp.log
LIBS=${LIBS:-libcep.so}
for lib in $LIBS; do
  CEP_LIB=$GRAFT_REPO_ROOT/flink-siddhi_amd/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_cf.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread >> gpurun_out/pytest_gpu.log 2>&1 || exit $?
done
for lib in $LIBS; do
  echo "== $lib" >> gpurun_out/cmp.log
  CEP_LIB=$GRAFT_REPO_ROOT/flink-siddhi_amd/$lib timeout -k 10 120 python bench.py --events 134217728 --steps 3 --warmup 1 --no-cpu 2>/dev/null | grep '^{' | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('serial', round(d['value']/1e9,2), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" >> gpurun_out/cmp.log || exit $?
  CEP_LIB=$GRAFT_REPO_ROOT/flink-siddhi_amd/$lib timeout -k 10 120 python bench.py --no-cpu 2>/dev/null | grep '^{' | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('overlap', round(d['value']/1e9,2), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" >> gpurun_out/cmp.log || exit $?
done
