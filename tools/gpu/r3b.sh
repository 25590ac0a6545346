# Pipelined MU solve: kernel tests, A/B bench (CNMF_SOLVE_PIPE=0/1), kernel trace.
set -e
export TMPDIR=/tmp
out=gpurun_out/r3b
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "solve or planes or nmf or mixed or refit" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_pipe.log 2>&1
CNMF_SOLVE_PIPE=0 timeout -k 10 120 python bench.py > $out/bench_nopipe.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/bench_grid.log 2>&1
timeout -k 10 150 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 3 --warmup 2 > $out/prof.log 2>&1
echo done
