# Iteration loop on the GPU box: parity tests, phase stamps, bench.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
CEP_STAMPS=1 timeout -k 10 300 python bench.py --events 67108864 --steps 2 --warmup 1 --no-cpu > gpurun_out/stamps.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --events 134217728 --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_serial.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1 || exit $?
exit 0
