# KL on fp16 counts: op tests, solver tests, KL bench (counts on / off)
set -e
export TMPDIR=/tmp
out=gpurun_out/r3t
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "beta or kl or bf16 or nmf_batch_gpu" > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
CNMF_KL_FP16_COUNTS=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_fp32x.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl2.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 > $out/prof_kl.log 2>&1
echo done
