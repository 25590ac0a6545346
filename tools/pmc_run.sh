#!/bin/bash
# Hardware-counter passes (one metric per rocprofv3 run, never combined with API tracing)
# over the Frobenius bench and the KL bench.  usage (via gpurun): bash tools/pmc_run.sh <tag>
set -o pipefail
TAG=${1:-pmc}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
for M in ${PMC_METRICS:-MfmaUtil LdsBankConflict OccupancyPercent MemUnitStalled VALUBusy}; do
  timeout -k 10 200 rocprofv3 --pmc $M --output-format csv -d gpurun_out/pmc_${TAG}/frob_$M -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/pmc_${TAG}_frob_$M.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc $M --output-format csv -d gpurun_out/pmc_${TAG}/kl_$M -o run -- python bench.py --steps 1 --warmup 0 --beta-loss kullback-leibler --n-iter 20 > gpurun_out/pmc_${TAG}_kl_$M.log 2>&1 || exit 1
done
