# XCD-aware slice-major pipe mapping A/B; then the r4e set
export TMPDIR=/tmp
out=gpurun_out/r4f
mkdir -p $out
CNMF_PIPE_MAP=1 timeout -k 10 400 python -u -m pytest tests/test_solve_pipe_gpu.py -x -q --timeout 120 --timeout-method thread > $out/pytest_map1.log 2>&1 || { echo PYTEST_MAP1_FAILED; tail -30 $out/pytest_map1.log; exit 1; }
for m in 0 1; do
  CNMF_PIPE_MAP=$m timeout -k 10 120 python bench.py > $out/bench_map$m.log 2>&1 &&
  CNMF_PIPE_MAP=$m timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_map$m.log 2>&1 &&
  CNMF_PIPE_MAP=$m timeout -k 10 200 python tools/pipe_stamp_probe.py --k 20 > $out/stamps_k20_map$m.log 2>&1 || exit 1
done &&
bash tools/gpu/r4e.sh
echo rc=$?
