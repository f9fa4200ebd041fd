# Bench with and without per-kernel timer events (profile 1 / 0) and the
# kernel trace's inter-kernel gaps.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CEP_PROFILE=1 timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_p1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/bench_p0.log 2>&1 || exit $?
python - <<'PY'
import json
for f in ("gpurun_out/bench_p1.log", "gpurun_out/bench_p0.log"):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, "%.2f G ev/s" % (d["value"] / 1e9), d["ms_per_step"], {k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
bash scripts/gpu_trace.sh > /dev/null && python scripts/trace_gaps.py | head -6
