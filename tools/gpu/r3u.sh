# KL fp16 counts: both sides / W side only / off
set -e
export TMPDIR=/tmp
out=gpurun_out/r3u
mkdir -p $out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fp16_count or online_kl_matches" > $out/pytest.log 2>&1
for v in 1 w 0 1 w; do CNMF_KL_FP16_COUNTS=$v timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_$v.log 2>&1; grep -h '^{' $out/bench_kl_$v.log >> $out/all.log; done
echo done
