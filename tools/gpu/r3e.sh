# Coop workspace reserved before capture; compaction-fraction A/B; e2e pipeline.
set -e
export TMPDIR=/tmp
out=gpurun_out/r3e
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused or pipe or graph or nmf or mixed" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
CNMF_COMPACT_FRAC_SMALL=0.5 timeout -k 10 120 python bench.py > $out/bench_cf50.log 2>&1
CNMF_COMPACT_FRAC_SMALL=0.35 timeout -k 10 120 python bench.py > $out/bench_cf35.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/bench_grid.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $out/prof.log 2>&1
echo done
