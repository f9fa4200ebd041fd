set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/sweep.log
for cfg in ${CFGS:-"--chunk 16777216"}; do
  echo "== $cfg" >> gpurun_out/sweep.log
  timeout -k 10 120 python bench.py --events 134217728 --steps 3 --warmup 1 --no-cpu $cfg 2>/dev/null | grep '^{' | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('serial',round(d['value']/1e9,2), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" >> gpurun_out/sweep.log || exit $?
  timeout -k 10 120 python bench.py --events 134217728 --steps 3 --warmup 1 --no-cpu $cfg 2>/dev/null | grep '^{' | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print('overlap',round(d['value']/1e9,2), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" >> gpurun_out/sweep.log || exit $?
done
