#!/bin/bash
# The round's measurement set (results under gpurun_out/, copied to profiles/
# by hand): bench lines for every workload, rocprofv3 kernel stats, PMC
# passes, the GPU test suite.  Each step has its own time limit
# (scripts/gpu_steps.sh).  usage: scripts/gpu_round.sh 1|2|3 [round tag, e.g. r04]
cd "${GRAFT_REPO_ROOT:-/root/repo}"
R="$PWD"
PART=${1:-1}
RN=${2:-r04}
P="rocprofv3 --kernel-trace --stats --output-format csv -o run -d"
if [ "$PART" = 1 ]; then
scripts/gpu_steps.sh \
  "450 gputest python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "300 b3 python -u bench.py" \
  "300 s3 cd /tmp && $P $R/gpurun_out/s3 -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-parity" \
  "300 b5 python -u bench.py --workload config5" \
  "200 s5 cd /tmp && $P $R/gpurun_out/s5 -- python3 $R/bench.py --workload config5 --steps 3 --warmup 1 --no-cpu --no-parity"
elif [ "$PART" = 2 ]; then
scripts/gpu_steps.sh \
  "200 b2 python -u bench.py --workload filter" \
  "200 s2 cd /tmp && $P $R/gpurun_out/s2 -- python3 $R/bench.py --workload filter --steps 3 --warmup 1 --no-cpu --no-parity" \
  "300 bz python -u bench.py --keys-dist zipf" \
  "200 bdo python -u bench.py --deliver --ordered --no-cpu --no-parity" \
  "200 bd python -u bench.py --deliver --no-cpu --no-parity" \
  "200 bdseq python -u bench.py --deliver --ordered --with-seq --no-cpu --no-parity" \
  "200 rank2 env CEP_DIST_BACKEND=gloo python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 2 --no-cpu" \
  "200 bh python -u bench.py --ingest host --no-cpu --no-parity" \
  "200 sdo cd /tmp && $P $R/gpurun_out/sdo -- python3 $R/bench.py --deliver --ordered --steps 3 --warmup 1 --no-cpu --no-parity"
else
scripts/gpu_steps.sh \
  "400 pmc3 bash scripts/gpu_pmc.sh ${RN}_pmc_config3.json" \
  "300 pmc5 env BENCH_ARGS='--workload config5' PMC_EVENTS=16777216 bash scripts/gpu_pmc.sh ${RN}_pmc_config5.json" \
  "300 pmcf env BENCH_ARGS='--workload filter' PMC_EVENTS=100000000 bash scripts/gpu_pmc.sh ${RN}_pmc_filter.json" \
  "120 calibf cd /tmp && timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/gpurun_out/calib -o calib -- python3 $R/scripts/filter_calib.py"
fi
