# KL column tiles per wave A/B (CT 1 vs 2), no retry back-edge; quick beta tests first
set -e
export TMPDIR=/tmp
out=gpurun_out/r3l
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "bf16 or kl_fp16 or online_kl_matches or online_beta" > $out/pytest.log 2>&1
CNMF_BP_KL_CT=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_ct1.log 2>&1
CNMF_BP_KL_CT=2 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_ct2.log 2>&1
CNMF_BP_KL_CT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 > $out/prof_kl.log 2>&1
echo done
