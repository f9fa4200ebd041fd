# Kernel trace of the default bench (3 timed steps): per-kernel stats plus the
# raw trace for gap analysis (scripts/trace_gaps.py).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/trace" -o run --output-format csv -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$R/gpurun_out/trace.txt" 2>&1 || exit $?
find "$R/gpurun_out/trace" -name "*.csv" | head
