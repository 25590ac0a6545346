# e2e pipeline bench twice (variance) + cProfile, and the 1M config with a warmup step.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e1.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_cprofile.txt > $out/e2e2.log 2>&1
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 25 --steps 2 --warmup 1 > $out/large_1M.log 2>&1
