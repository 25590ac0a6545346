# large-N configs at HEAD: DP emulated rank at 10M x 5k (kernel summary), 1M x 2k, 10M x 5k single GPU
export TMPDIR=/tmp
out=gpurun_out/r4u
mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_emu8_10m -o run --output-format csv -- python3 tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 25 --dp --emulate-world 8 --planes-only --steps 1 > $out/emu8_10m.log 2>&1 &&
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --steps 2 --warmup 1 > $out/large_1m_r100.log 2>&1 &&
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --dp --emulate-world 8 --steps 2 --warmup 1 > $out/emu8_1m.log 2>&1 &&
timeout -k 10 600 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 8 --planes-only --steps 1 > $out/large_10m.log 2>&1
echo rc=$?
