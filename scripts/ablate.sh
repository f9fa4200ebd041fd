set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; : > gpurun_out/ablate.log
for ab in ${ABL:-0 1 2 3}; do
  echo "== ablate $ab" >> gpurun_out/ablate.log
  CEP_ABLATE=$ab timeout -k 10 120 python bench.py --events 134217728 --steps 3 --warmup 1 --no-cpu 2>/dev/null | grep '^{' | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());print(round(d['value']/1e9,2), {k:round(v['avg_us'],1) for k,v in d['kernels'].items()})" >> gpurun_out/ablate.log || exit $?
done
