#!/bin/bash
# Hardware-counter passes over the Frobenius bench only (one metric per rocprofv3 run,
# kernel trace only, no API tracing).  usage (via gpurun): bash tools/pmc_frob.sh <tag>
set -o pipefail
TAG=${1:-pmcf}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in ${PMC_METRICS:-MfmaUtil OccupancyPercent LdsBankConflict VALUBusy}; do
  timeout -k 10 120 rocprofv3 --pmc $M --output-format csv -d gpurun_out/pmc_${TAG}/frob_$M -o run -- python bench.py --steps 1 --warmup 1 > gpurun_out/pmc_${TAG}_frob_$M.log 2>&1 || exit 1
done
