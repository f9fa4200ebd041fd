# A/B on the GPU box: parity tests, then the default bench with the current
# build and with an env switch (ENV_B, e.g. CEP_CFPART=0) for comparison.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then tail -30 gpurun_out/pytest_gpu.log; exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_a.log 2>&1 || exit $?
env ${ENV_B:-CEP_NOTHING=1} timeout -k 10 300 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench_b.log 2>&1 || exit $?
tail -1 gpurun_out/pytest_gpu.log
python - <<'PY'
import json
for f in ("gpurun_out/bench_a.log", "gpurun_out/bench_b.log"):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    print(f, "%.2f G ev/s" % (d["value"] / 1e9), {k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
