# sparse KL: two replicates per workgroup on the spectra side
export TMPDIR=/tmp
out=gpurun_out/r4x
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "kl" -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for d in 0.08 0.15; do
  for pr in 1 0; do
    CNMF_KL_PAIR=$pr timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_p$pr.log 2>&1 || exit 1
  done
done
echo rc=$?
