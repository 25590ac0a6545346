# Wide-K (65..128) matrix-core MU solve + Gram tests; conflict-free beta panel strides: beta tests,
# KL bench (fp16 counts on/w/off), usage-kernel occupancy A/B (CNMF_BP_OCC=3)
set -e
export TMPDIR=/tmp
out=gpurun_out/r3w
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "wmfma or wide or gram or refit_wide" > $out/pytest_wide.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "beta or kl or bf16" > $out/pytest_beta.log 2>&1
for v in 1 w 0; do CNMF_KL_FP16_COUNTS=$v timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_$v.log 2>&1; done
for v in 1 w; do CNMF_BP_OCC=3 CNMF_KL_FP16_COUNTS=$v timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_occ3_$v.log 2>&1; done
echo done
