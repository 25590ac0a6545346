# round 4 first pass: K > 16 pipelined solve tests, HEAD-before (_before/, built from
# 39fc4ce) vs after benches at K = 20 / 30, headline, kernel summaries
export TMPDIR=/tmp
out=gpurun_out/r4a
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_kernels_gpu.py -k "pipe or fused or gram_of" -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
(cd _before && timeout -k 10 200 python bench.py --k 20 --steps 5 --warmup 2 > ../$out/before_k20.log 2>&1) &&
(cd _before && timeout -k 10 200 python bench.py --k 30 --steps 5 --warmup 2 > ../$out/before_k30.log 2>&1) &&
timeout -k 10 200 python bench.py --k 20 --steps 5 --warmup 2 > $out/after_k20.log 2>&1 &&
timeout -k 10 200 python bench.py --k 30 --steps 5 --warmup 2 > $out/after_k30.log 2>&1 &&
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof20 -o run --output-format csv -- python3 bench.py --k 20 --steps 3 --warmup 1 > $out/prof20.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof30 -o run --output-format csv -- python3 bench.py --k 30 --steps 3 --warmup 1 > $out/prof30.log 2>&1 &&
(cd _before && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d ../$out/prof20b -o run --output-format csv -- python3 bench.py --k 20 --steps 3 --warmup 1 > ../$out/prof20b.log 2>&1)
echo rc=$?
tail -3 $out/*.log
