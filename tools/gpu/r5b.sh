# streaming (continuous batching) first light: pipe / stream tests, headline stream vs batch, K=20
export TMPDIR=/tmp
out=gpurun_out/r5b
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_solve_pipe_gpu.py -x -v --timeout 170 --timeout-method thread -k stream > $out/pytest_stream.log 2>&1
echo pytest_rc=$?
timeout -k 10 200 python bench.py > $out/bench_stream.log 2>&1 &&
timeout -k 10 200 python bench.py --schedule batch > $out/bench_batch.log 2>&1 &&
timeout -k 10 200 python bench.py --live 100 > $out/bench_stream100.log 2>&1 &&
timeout -k 10 200 python bench.py --k 20 > $out/k20_stream.log 2>&1 &&
timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 6 --warmup 2 > $out/grid_stream.log 2>&1
echo rc=$?
tail -n 1 $out/*.log
