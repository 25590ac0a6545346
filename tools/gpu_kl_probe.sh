# KL kernel probe: per-call kernel times and the per-dispatch histogram of the KL bench.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 120 python tools/beta_probe.py > $out/beta_probe.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl -o run -- python3 bench.py --beta-loss kullback-leibler --steps 1 --warmup 1 > $out/prof_kl.log 2>&1
python tools/kernel_hist.py $out/prof_kl beta_h_kernel beta_w_kernel beta_w_update > $out/kl_hist.txt 2>&1
