#!/bin/bash
# Counter passes over the headline bench (one counter group per rocprofv3 run, kernel
# trace only -- never combined with API / system tracing).  usage: bash
# tools/gpu/pmc_headline.sh TAG [bench args]; summary: python tools/pmc_summary.py
# gpurun_out/TAG
export TMPDIR=/tmp
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
for M in ${PMC_METRICS:-MfmaUtil VALUBusy LdsBankConflict MemUnitStalled OccupancyPercent}; do
  timeout -s KILL 120 rocprofv3 --pmc $M --output-format csv -d "$out/$M" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-stream-value "$@" > "$out/$M.log" 2>&1 || {
    echo "PMC $M failed"; tail -5 "$out/$M.log"; exit 1; }
  echo "pmc $M ok"
done
