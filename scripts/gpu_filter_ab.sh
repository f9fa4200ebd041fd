set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_reorder.py tests/test_gpu_agg.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --workload filter --no-cpu > gpurun_out/bf_a.log 2>&1 || exit $?
CEP_FILTER1=1 timeout -k 10 300 python bench.py --workload filter --no-cpu > gpurun_out/bf_b.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/bf_a.log", "gpurun_out/bf_b.log"):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, "%.2f G ev/s" % (d["value"] / 1e9), d["roofline"]["frac"], {k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
