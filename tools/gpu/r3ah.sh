# GEMM gate (speculative last pass skips its GEMMs) + async init seeds + parallel k-means accumulation:
# tests, headline A/B, grid, pass trace, Harmony 500k
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ah
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused or graph or mixed_k or nmf_batch_gpu or concurrent or split_gemm or gemm or philox or kmeans or harmony" > $out/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py > $out/bench_on_$i.log 2>&1
  CNMF_GEMM_GATE=0 timeout -k 10 120 python bench.py > $out/bench_off_$i.log 2>&1
done
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/prof.log 2>&1
timeout -k 10 450 python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony.log 2>&1
echo done
