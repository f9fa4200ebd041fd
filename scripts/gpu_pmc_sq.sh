# One PMC pass of SQ instruction counters (no tracing domains).
set -u
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
ARGS="--events ${PMC_EVENTS:-67108864} --steps 2 --warmup 1 --no-cpu ${BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d "$R/gpurun_out/pmcsq" -o "pass" -- python3 "$R/bench.py" $ARGS > "$R/gpurun_out/pmcsq.log" 2>&1 || exit $?
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmcsq" "$R/gpurun_out/pmcsq_summary.json" > "$R/gpurun_out/pmcsq_summary.txt" 2>&1
exit 0
