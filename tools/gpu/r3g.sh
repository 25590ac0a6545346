# e2e after native prepare stats; 10M x 5k planes-only kernel summary; headline bench with
# sweep counts; KL bench baseline; MfmaUtil / VALUBusy PMC of the headline step.
set -e
export TMPDIR=/tmp
out=gpurun_out/r3g
mkdir -p $out
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_10M -o run --output-format csv -- python3 tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 8 --planes-only > $out/large_10M_prof.log 2>&1
for M in MfmaUtil VALUBusy OccupancyPercent; do
timeout -s KILL 120 rocprofv3 --pmc $M --output-format csv -d $out/pmc_$M -o run -- python3 bench.py --steps 1 --warmup 1 > $out/pmc_$M.log 2>&1
done
echo done
