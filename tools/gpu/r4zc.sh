# secondary configurations at HEAD (end of round 4)
export TMPDIR=/tmp
out=gpurun_out/r4zc
mkdir -p $out
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1 &&
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density 0.08 --steps 3 --warmup 1 > $out/kl_d08.log 2>&1 &&
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/kl.log 2>&1 &&
timeout -k 10 200 python bench.py --float-input --steps 10 --warmup 3 > $out/float.log 2>&1 &&
timeout -k 10 200 python bench.py --k 50 --steps 3 --warmup 1 > $out/k50.log 2>&1 &&
timeout -k 10 200 python bench.py --k 100 --steps 2 --warmup 1 > $out/k100.log 2>&1 &&
timeout -k 10 200 python bench.py --k 128 --steps 2 --warmup 1 > $out/k128.log 2>&1 &&
timeout -k 10 200 python bench.py --algo hals --steps 10 --warmup 3 > $out/hals.log 2>&1 &&
timeout -k 10 600 python tools/bench_harmony.py > $out/harmony.log 2>&1
echo rc=$?
