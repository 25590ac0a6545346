# round-5 baseline at HEAD: headline, K=20, K=30, K=20 kernel summary
export TMPDIR=/tmp
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 150 python bench.py --k 20 > $out/k20.log 2>&1 &&
timeout -k 10 150 python bench.py --k 30 > $out/k30.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_k20 -o run --output-format csv -- python3 bench.py --k 20 --steps 4 --warmup 2 > $out/prof_k20.log 2>&1
echo rc=$?
