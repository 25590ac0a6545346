# library pre-warm during factorize (e2e first-stage costs); graph tests with thread-local capture
export TMPDIR=/tmp
out=gpurun_out/r4zd
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_solve_pipe_gpu.py tests/test_pipeline_gpu.py -k "graph or replay or fused or pipeline or k_selection or resident" -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for rep in 1 2 3; do
  for w in 0 1; do
    CNMF_PREWARM=$w timeout -k 10 300 python tools/bench_e2e.py > $out/e2e_w${w}_$rep.log 2>&1 || exit 1
  done
done
echo rc=$?
