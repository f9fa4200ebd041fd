set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
i=0
while read -r args; do
  timeout -k 10 300 python bench.py --no-cpu $args > gpurun_out/sw_$i.log 2>&1 || exit $?
  python - "$i" "$args" <<'PY'
import json, sys
d = json.loads([l for l in open("gpurun_out/sw_%s.log" % sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "%.2f G ev/s" % (d["value"] / 1e9), {k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
  i=$((i+1))
done <<< "${SWEEP:---chunk 33554432}"
