# resident mirror / pinned D2H / Harmony stages; KL CSR crossover (forced)
export TMPDIR=/tmp
out=gpurun_out/r4e
mkdir -p $out
timeout -k 10 500 python -u -m pytest tests/test_pipeline_gpu.py tests/test_preprocess.py -x -q --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 120 python tools/d2h_probe.py > $out/d2h.log 2>&1 &&
for d in 0.15 0.25 0.35; do
  CNMF_KL_SPARSE=1 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_sparse.log 2>&1 &&
  CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_dense.log 2>&1 || exit 1
done &&
timeout -k 10 600 python tools/bench_harmony.py --profile-stages $out/hstage > $out/harmony.log 2>&1
echo rc=$?
