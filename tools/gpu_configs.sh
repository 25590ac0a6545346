# BASELINE configs on one MI355X with the current code: e2e PBMC-scale pipeline (config 2),
# 1M x 2k K=10 (config 3, this GPU's 25 of 200 replicates), Harmony 500k (config 5),
# 10M x 5k K=20 whole matrix on one GPU (config 4 shape).
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 25 > $out/large_1M.log 2>&1
timeout -k 10 400 python tools/bench_harmony.py > $out/harmony.log 2>&1
timeout -k 10 600 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 8 > $out/large_10M.log 2>&1
