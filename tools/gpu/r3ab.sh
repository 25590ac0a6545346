# Harmony reduce kernel one wave per (b, k): tests + 500k e2e; 1M x 2k K=10 refresh (25 and 100 replicates)
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ab
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "harmony or preprocess" > $out/pytest.log 2>&1
timeout -k 10 450 python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony.log 2>&1
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 25 --steps 2 --warmup 1 > $out/large_1M_r25.log 2>&1
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --steps 2 --warmup 1 > $out/large_1M_r100.log 2>&1
echo done
