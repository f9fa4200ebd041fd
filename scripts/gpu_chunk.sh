set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_cf.py tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/pytest_gpu.log; exit 1; }
for c in 16777216 33554432; do
  timeout -k 10 300 python bench.py --no-cpu --chunk $c > gpurun_out/chunk_$c.log 2>&1 || exit $?
done
tail -1 gpurun_out/pytest_gpu.log
python - <<'PY'
import json
for c in (16777216, 33554432):
    d = json.loads([l for l in open("gpurun_out/chunk_%d.log" % c) if l.startswith("{")][-1])
    print("chunk", c, "%.2f G ev/s" % (d["value"] / 1e9), {k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
