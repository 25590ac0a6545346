# kernel summaries: Harmony + cNMF (500k cells, 4 covariates) and 10M x 5k planes-only
set -e
export TMPDIR=/tmp
out=gpurun_out/r3q
mkdir -p $out
timeout -k 10 450 rocprofv3 --kernel-trace --stats -d $out/prof_harmony -o run --output-format csv -- python3 tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony.log 2>&1
timeout -k 10 450 rocprofv3 --kernel-trace --stats -d $out/prof_10M -o run --output-format csv -- python3 tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 8 --planes-only > $out/large_10M.log 2>&1
echo done
