# PMC passes (one counter group per pass; never combined with tracing domains),
# then scripts/pmc_summary.py.  usage: scripts/gpu_pmc.sh [out.json]
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
ARGS="--events ${PMC_EVENTS:-67108864} --steps 2 --warmup 1 --no-cpu --no-parity ${BENCH_ARGS:-}"
# PMC_SCRIPT / PMC_SCRIPT_ARGS: profile another program (e.g. scripts/route_padded_bench.py)
SCRIPT="${PMC_SCRIPT:-$R/bench.py}"
if [ -n "${PMC_SCRIPT:-}" ]; then ARGS="${PMC_SCRIPT_ARGS:-}"; fi
GROUPS_DEFAULT=("FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum")
if [ -n "${PMC_GROUPS:-}" ]; then IFS='|' read -ra GROUPS_DEFAULT <<< "$PMC_GROUPS"; fi
i=0
rm -rf "$R/gpurun_out/pmc"
for grp in "${GROUPS_DEFAULT[@]}"; do
  i=$((i+1))
  echo "pass $i: $grp"
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d "$R/gpurun_out/pmc" -o "pass$i" -- python3 "$SCRIPT" $ARGS > "$R/gpurun_out/pmc_pass$i.txt" 2>&1 || exit $?
done
python3 "$R/scripts/pmc_summary.py" "$R/gpurun_out/pmc" "$R/gpurun_out/${1:-pmc_summary.json}"
exit 0
