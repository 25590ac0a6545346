# KL / IS native to K = 64 / 56 and the fused Harmony round: kernel + solver tests,
# KL bench at K=48 and K=10, Harmony 500k end to end
export TMPDIR=/tmp
out=gpurun_out/r5h
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_preprocess.py -x -v --timeout 170 --timeout-method thread -k "beta or harmony" > $out/pytest_beta.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest_beta.log | head -30; exit 1; }
tail -2 $out/pytest_beta.log
timeout -k 10 300 python bench.py --beta-loss kullback-leibler --k 48 --steps 3 --warmup 1 > $out/kl48.log 2>&1 && tail -n 1 $out/kl48.log | cut -c1-250 &&
timeout -k 10 300 python bench.py --beta-loss kullback-leibler --steps 5 --warmup 1 > $out/kl10.log 2>&1 && tail -n 1 $out/kl10.log | cut -c1-250 &&
timeout -k 10 600 python tools/bench_harmony.py > $out/harmony.log 2>&1 && tail -n 1 $out/harmony.log
echo rc=$?
