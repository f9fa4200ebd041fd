#!/bin/bash
# Diagnostics: run one test under several CEP_ABLATE values (and the k_cfwalk
# build); a time limit or crash stops the run.
# usage: scripts/bisect_ablate.sh <test id> <ablate values...>
t=$1; shift
mkdir -p gpurun_out
for ab in "$@" old; do
  if [ "$ab" = old ]; then env="CEP_CF_WALK=1"; else env="CEP_ABLATE=$ab"; fi
  env $env timeout -k 10 120 python -u -m pytest -x -q --timeout 100 --timeout-method thread "$t" > gpurun_out/ab_$ab.txt 2>&1
  rc=$?
  echo "== $env rc=$rc: $(tail -1 gpurun_out/ab_$ab.txt)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
