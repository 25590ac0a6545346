# Fused step v2 (slab rounds, device coop generation, slab cap): tests, A/B benches, trace.
set -e
export TMPDIR=/tmp
out=gpurun_out/r3d
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused or pipe or solve or planes or nmf or mixed or refit or gemm or graph" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_fused.log 2>&1
CNMF_GRAPHS=0 timeout -k 10 120 python bench.py > $out/bench_nographs.log 2>&1
CNMF_FUSED_STEP=0 timeout -k 10 120 python bench.py > $out/bench_unfused.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/bench_grid.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $out/prof.log 2>&1
echo done
