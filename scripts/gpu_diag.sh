#!/bin/bash
# Round-3 diagnostics set: config-5 cost split + walk phase stamps, rocprofv3
# kernel stats of config 5 and of ordered delivery, PMC of config 5 and the
# filter.  Each step under its own time limit (scripts/gpu_steps.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
P="rocprofv3 --kernel-trace --stats --output-format csv -o run -d"
scripts/gpu_steps.sh \
  "150 optest python -u -m pytest tests/test_gpu_operator.py -v --timeout 120 --timeout-method thread" \
  "200 split python -u scripts/config5_split.py" \
  "150 stamps5 env CEP_STAMPS=1 python -u bench.py --workload config5 --no-cpu --no-parity --steps 2" \
  "200 s5 cd /tmp && $P $R/gpurun_out/s5 -- python3 $R/bench.py --workload config5 --steps 3 --warmup 1 --no-cpu --no-parity" \
  "200 sdo cd /tmp && $P $R/gpurun_out/sdo -- python3 $R/bench.py --deliver --ordered --steps 3 --warmup 1 --no-cpu --no-parity" \
  "300 pmc5 env BENCH_ARGS='--workload config5' PMC_EVENTS=16777216 bash scripts/gpu_pmc.sh r03_pmc_config5.json" \
  "300 pmcf env BENCH_ARGS='--workload filter' PMC_EVENTS=100000000 bash scripts/gpu_pmc.sh r03_pmc_filter.json"
