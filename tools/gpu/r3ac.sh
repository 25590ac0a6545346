# Harmony + cNMF 500k: host cProfile of every stage
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ac
mkdir -p $out
timeout -k 10 500 python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 --profile $out/prof.harmony.txt --profile-stages $out/prof > $out/harmony.log 2>&1
echo done
