# Frobenius path: GEMM/solve/NMF GPU tests, bench, kernel-trace profile of the bench.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm or solve or nmf or concurrent or graph or coop" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
python tools/prof_summary.py $out/prof/run_results.db --top 20 > $out/kernels.txt 2>&1 || true
