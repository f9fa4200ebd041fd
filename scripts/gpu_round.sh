#!/bin/bash
# The round's measurement set (results under gpurun_out/, copied to profiles/
# by hand): bench lines for every workload, rocprofv3 kernel stats of the
# config-3 / config-2 / Zipf benches, PMC passes of config 3, the 2-rank
# rehearsal.  Each step has its own time limit (scripts/gpu_steps.sh).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
PART=${1:-1}
P="rocprofv3 --kernel-trace --stats --output-format csv -o run -d"
if [ "$PART" = 1 ]; then
scripts/gpu_steps.sh \
  "300 b3 python -u bench.py" \
  "300 s3 cd /tmp && $P $GRAFT_REPO_ROOT/gpurun_out/s3 -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-parity" \
  "200 b2 python -u bench.py --workload filter" \
  "200 s2 cd /tmp && $P $GRAFT_REPO_ROOT/gpurun_out/s2 -- python3 $GRAFT_REPO_ROOT/bench.py --workload filter --steps 3 --warmup 1 --no-cpu --no-parity" \
  "300 bz python -u bench.py --keys-dist zipf" \
  "300 sz cd /tmp && $P $GRAFT_REPO_ROOT/gpurun_out/sz -- python3 $GRAFT_REPO_ROOT/bench.py --keys-dist zipf --steps 3 --warmup 1 --no-cpu --no-parity"
else
scripts/gpu_steps.sh \
  "300 b5 python -u bench.py --workload config5" \
  "200 bh python -u bench.py --ingest host --no-cpu --no-parity --deliver" \
  "600 pmc bash scripts/gpu_pmc.sh r02_pmc.json" \
  "600 multi bash scripts/gpu_multi_rehearsal.sh"
fi
