# KL: fp16-numerator dense kernels + CSR kernels; tests, benches (dense 47 %, 15 % sparse vs dense), trace
set -e
export TMPDIR=/tmp
out=gpurun_out/r3j
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "beta or kl or bf16 or nmf_batch_gpu" > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 --density 0.15 > $out/bench_kl_d15_sparse.log 2>&1
CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 --density 0.15 > $out/bench_kl_d15_dense.log 2>&1
CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_d47_sparse.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof_kl -o run -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 > $out/prof_kl.log 2>&1
CNMF_KL_SPARSE=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof_kl_d15 -o run -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 --density 0.15 > $out/prof_kl_d15.log 2>&1
echo done
