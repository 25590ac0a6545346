# occupancy cap A/B (CNMF_PIPE_MAXWG) at K = 10 / 20 / 30
export TMPDIR=/tmp
out=gpurun_out/r4p
mkdir -p $out
CNMF_PIPE_MAXWG=3 timeout -k 10 300 python -u -m pytest tests/test_solve_pipe_gpu.py -x -q --timeout 120 --timeout-method thread -k "bitwise or fused" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for m in 3 0; do
  CNMF_PIPE_MAXWG=$m timeout -k 10 120 python bench.py > $out/bench_m$m.log 2>&1;
  CNMF_PIPE_MAXWG=$m timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_m$m.log 2>&1;
  CNMF_PIPE_MAXWG=$m timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30_m$m.log 2>&1
done
echo rc=$?
