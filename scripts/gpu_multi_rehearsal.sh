# Two ranks sharing the box's single GPU (gloo, host-staged exchange): exercises
# bench.py's multi-GPU shuffle path end to end.  The real N>1 runs use RCCL.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
CEP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --events 16777216 --steps 2 --warmup 1 \
  --no-cpu > gpurun_out/multi_rehearsal.txt 2>&1
rc=$?
[ $rc -ne 0 ] && { tail -20 gpurun_out/multi_rehearsal.txt; exit $rc; }
CEP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --events 16777216 --steps 2 --warmup 1 \
  --no-cpu --ingest prepartitioned > gpurun_out/multi_rehearsal_pre.txt 2>&1 || { tail -20 gpurun_out/multi_rehearsal_pre.txt; exit 1; }
CEP_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --workload config5 --events 4194304 --steps 2 \
  --warmup 1 > gpurun_out/multi_rehearsal_c5.txt 2>&1 || { tail -20 gpurun_out/multi_rehearsal_c5.txt; exit 1; }
grep -h '^{' gpurun_out/multi_rehearsal.txt gpurun_out/multi_rehearsal_pre.txt gpurun_out/multi_rehearsal_c5.txt | cut -c1-400
