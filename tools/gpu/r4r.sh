# wave-quantisation GEMM plan A/B
export TMPDIR=/tmp
out=gpurun_out/r4r
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "gemm or fused or slots or wide" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for w in 1 0; do
  CNMF_GEMM_WAVE_PLAN=$w timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_w$w.log 2>&1 &&
  CNMF_GEMM_WAVE_PLAN=$w timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30_w$w.log 2>&1 &&
  CNMF_GEMM_WAVE_PLAN=$w timeout -k 10 120 python bench.py --k 50 --steps 3 --warmup 1 > $out/k50_w$w.log 2>&1 &&
  CNMF_GEMM_WAVE_PLAN=$w timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_w$w.log 2>&1 || exit 1
done &&
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
echo rc=$?
