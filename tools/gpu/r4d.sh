# f0 deferral + prologue: tests, stamps, bench; KL crossover; Harmony stage profiles
export TMPDIR=/tmp
out=gpurun_out/r4d
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20.log 2>&1 &&
timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30.log 2>&1 &&
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 10 > $out/stamps_k10.log 2>&1 &&
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 20 > $out/stamps_k20.log 2>&1 &&
for d in 0.15 0.25; do
  timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_sparse.log 2>&1 &&
  CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_dense.log 2>&1 || exit 1
done &&
timeout -k 10 600 python tools/bench_harmony.py --profile $out/harmony_prof.txt --profile-stages $out/hstage > $out/harmony.log 2>&1
echo rc=$?
