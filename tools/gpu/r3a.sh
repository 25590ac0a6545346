# Round-3 first GPU pass: xGMI memory-kind test, headline bench, kernel trace of the bench.
set -e
export TMPDIR=/tmp
out=gpurun_out/r3a
mkdir -p $out
timeout -k 10 240 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 120 --timeout-method thread > $out/pytest_xgmi.log 2>&1 || echo "xgmi tests failed rc=$?"
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/bench_grid.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $out/prof.log 2>&1
echo done
