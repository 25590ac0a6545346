# KL online MU: kernel trace of the headline KL bench (GPU busy vs idle per kernel family)
set -e
export TMPDIR=/tmp
out=gpurun_out/r3h
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof_kl -o run -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 > $out/prof_kl.log 2>&1
echo done
