# wide solve variant rule (bf16 at K%32==0) + CSR column stats unrolled: tests, K=100/128 benches, Harmony 500k trace
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ag
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_sparse_ops.py -x -q --timeout 120 --timeout-method thread -k "wmfma or wide or refit_wide or csr or colstats or sparse or mean_var" > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --k 100 --steps 3 --warmup 1 > $out/bench_k100.log 2>&1
timeout -k 10 200 python bench.py --k 128 --steps 3 --warmup 1 > $out/bench_k128.log 2>&1
timeout -k 10 450 rocprofv3 --kernel-trace --stats -d $out/prof_harmony -o run --output-format csv -- python3 tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony_prof.log 2>&1
echo done
