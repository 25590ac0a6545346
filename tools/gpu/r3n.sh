# sparse KL with LDS-staged S^T: tests + 15 % bench sparse vs dense
set -e
export TMPDIR=/tmp
out=gpurun_out/r3n
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "sparse_kl or kl_sparse" > $out/pytest.log 2>&1
CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 --density 0.15 > $out/bench_kl_d15_sparse.log 2>&1
CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 --density 0.15 > $out/bench_kl_d15_dense.log 2>&1
CNMF_KL_SPARSE=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl_d15 -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 --density 0.15 > $out/prof_kl_d15.log 2>&1
echo done
