# stamps compiled out, per-launch XCD map, fused gpart rounds; D2H, KL crossover, Harmony
export TMPDIR=/tmp
out=gpurun_out/r4h
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20.log 2>&1 &&
timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30.log 2>&1 &&
CNMF_PIPE_MAP=0 timeout -k 10 120 python bench.py > $out/bench_map0.log 2>&1 &&
timeout -k 10 120 python tools/d2h_probe.py > $out/d2h.log 2>&1 &&
for d in 0.15 0.25 0.35; do
  CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_sparse.log 2>&1 &&
  CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_dense.log 2>&1 || exit 1
done &&
timeout -k 10 600 python tools/bench_harmony.py --profile-stages $out/hstage > $out/harmony.log 2>&1
echo rc=$?
