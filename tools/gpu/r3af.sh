# split-bf16 Gram apply for the wide MU solve (K 65..128): tests (both variants), K=100/128 benches, kernel summary
set -e
export TMPDIR=/tmp
out=gpurun_out/r3af
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wmfma or wide or refit_wide" > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --k 100 --steps 3 --warmup 1 > $out/bench_k100.log 2>&1
timeout -k 10 200 python bench.py --k 128 --steps 3 --warmup 1 > $out/bench_k128.log 2>&1
CNMF_WIDE_SOLVE=fp32 timeout -k 10 200 python bench.py --k 128 --steps 3 --warmup 1 > $out/bench_k128_fp32.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_k128 -o run --output-format csv -- python3 bench.py --k 128 --steps 2 --warmup 1 > $out/prof_k128.log 2>&1
echo done
