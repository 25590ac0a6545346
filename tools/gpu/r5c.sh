# streaming v2 (staged refills, min-fill rounds): tests, stream vs batch, kernel trace
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_prepare_gpu.py -x -v --timeout 170 --timeout-method thread -k "stream or moment or prepare" > $out/pytest_stream.log 2>&1
echo pytest_rc=$?
timeout -k 10 200 python bench.py > $out/bench_stream.log 2>&1 &&
timeout -k 10 200 python bench.py --live 100 > $out/bench_stream100.log 2>&1 &&
CNMF_STREAM_MIN_FILL=1 timeout -k 10 200 python bench.py > $out/bench_stream_mf1.log 2>&1 &&
timeout -k 10 200 python bench.py --k 20 > $out/k20_stream.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_stream -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 > $out/prof_stream.log 2>&1
echo rc=$?
tail -n 1 $out/*.log
