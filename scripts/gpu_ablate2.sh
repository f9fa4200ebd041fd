set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for ab in 0 1 2 3; do
  CEP_ABLATE=$ab timeout -k 10 300 python bench.py --no-cpu --steps 3 > gpurun_out/ab_$ab.log 2>&1 || exit $?
done
python - <<'PY'
import json
for ab in range(4):
    d = json.loads([l for l in open("gpurun_out/ab_%d.log" % ab) if l.startswith("{")][-1])
    print("ablate", ab, "%.2f G ev/s" % (d["value"] / 1e9), {k: round(v["avg_us"], 1) for k, v in d["kernels"].items()})
PY
