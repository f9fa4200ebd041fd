# Per-kernel split of the shuffle sender (k_cfroute + gather) and an owner
# (rocprofv3 kernel trace of scripts/route_bench.py, world 8).
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"; mkdir -p "$R/gpurun_out"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/rprof" -o run -- python3 "$R/scripts/route_bench.py" ${WORLD:-8} > "$R/gpurun_out/route_bench.log" 2>&1
