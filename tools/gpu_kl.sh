# KL-loss bench + kernel profile + per-step inner-iteration counts.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl -o run -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 > $out/prof_kl.log 2>&1
