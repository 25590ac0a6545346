# slice-width A/B (K=10/20/30), K=20 kernel summary, KL routing test
export TMPDIR=/tmp
out=gpurun_out/r4i
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "kl_sparse" -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for c in 256 384 512; do
  CNMF_PIPE_SLICE_COLS=$c timeout -k 10 120 python bench.py > $out/bench_c$c.log 2>&1 &&
  CNMF_PIPE_SLICE_COLS=$c timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_c$c.log 2>&1 &&
  CNMF_PIPE_SLICE_COLS=$c timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30_c$c.log 2>&1 || exit 1
done &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_k20 -o run --output-format csv -- python3 bench.py --k 20 --steps 4 --warmup 2 > $out/prof_k20.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_k10 -o run --output-format csv -- python3 bench.py --steps 8 --warmup 2 > $out/prof_k10.log 2>&1
echo rc=$?
