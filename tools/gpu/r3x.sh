# flag copy on a side stream + no arena zeroing: headline A/B on one box, grid, per-pass trace
set -e
export TMPDIR=/tmp
out=gpurun_out/r3x
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused or graph or mixed_k or nmf_batch_gpu or concurrent" > $out/pytest.log 2>&1
for i in 1 2 3; do timeout -k 10 120 python bench.py > $out/bench_$i.log 2>&1; done
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/prof.log 2>&1
echo done
