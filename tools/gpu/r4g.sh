# device active list + XCD map A/B; resident mirror, D2H, KL crossover, Harmony stages
export TMPDIR=/tmp
out=gpurun_out/r4g
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_solve_pipe_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for m in 0 1; do
  CNMF_PIPE_MAP=$m timeout -k 10 120 python bench.py > $out/bench_map$m.log 2>&1 &&
  CNMF_PIPE_MAP=$m timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_map$m.log 2>&1 &&
  CNMF_PIPE_MAP=$m timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30_map$m.log 2>&1 &&
  CNMF_PIPE_MAP=$m timeout -k 10 200 python tools/pipe_stamp_probe.py --k 20 > $out/stamps_k20_map$m.log 2>&1 || exit 1
done &&
timeout -k 10 120 python tools/d2h_probe.py > $out/d2h.log 2>&1 &&
for d in 0.15 0.25 0.35; do
  CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_sparse.log 2>&1 &&
  CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_dense.log 2>&1 || exit 1
done &&
timeout -k 10 600 python tools/bench_harmony.py --profile-stages $out/hstage > $out/harmony.log 2>&1
echo rc=$?
