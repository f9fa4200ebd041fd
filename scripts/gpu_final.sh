# Round artifacts: GPU parity suite, smoke, default bench (with CPU baseline),
# rocprofv3 kernel stats of the bench, PMC passes.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$GRAFT_REPO_ROOT"
PROF=1 bash scripts/gpu_check.sh || { echo "gpu_check failed"; tail -20 gpurun_out/pytest_gpu.log; exit 1; }
bash scripts/gpu_pmc.sh || { echo "pmc failed"; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
cat gpurun_out/smoke.log | grep -v amdgpu.ids
grep '^{' gpurun_out/bench.log | cut -c1-300
