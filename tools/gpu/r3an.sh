# refresh the secondary configurations at HEAD: float input, K = 50 / 100 / 128, HALS, batch mode,
# sparse KL at 15 % density, 1M cells, 10M x 5k planes only, Harmony 500k
set -e
export TMPDIR=/tmp
out=gpurun_out/r3an
mkdir -p $out
timeout -k 10 120 python bench.py --float-input > $out/bench_float.log 2>&1
timeout -k 10 200 python bench.py --k 50 --steps 3 --warmup 1 > $out/bench_k50.log 2>&1
timeout -k 10 200 python bench.py --k 100 --steps 3 --warmup 1 > $out/bench_k100.log 2>&1
timeout -k 10 200 python bench.py --k 128 --steps 3 --warmup 1 > $out/bench_k128.log 2>&1
timeout -k 10 200 python bench.py --algo hals --steps 5 --warmup 2 > $out/bench_hals.log 2>&1
timeout -k 10 200 python bench.py --nmf-mode batch --steps 3 --warmup 1 > $out/bench_batch.log 2>&1
CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 --density 0.15 > $out/bench_kl_d15_sparse.log 2>&1
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --steps 2 --warmup 1 > $out/large_1M_r100.log 2>&1
timeout -k 10 400 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 8 --planes-only > $out/large_10M_planes.log 2>&1
timeout -k 10 450 python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony.log 2>&1
echo done
