set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CEP_STAMPS=1 timeout -k 10 300 python bench.py --events 67108864 --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-} > gpurun_out/stamps.log 2>&1
