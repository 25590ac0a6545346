# final validation at HEAD: xGMI tests, full GPU suite, smoke, headline + K=20 kernel summaries
export TMPDIR=/tmp
out=gpurun_out/r4zb
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 170 --timeout-method thread > $out/pytest_xgmi.log 2>&1 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_bench -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 > $out/prof_bench.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_k20 -o run --output-format csv -- python3 bench.py --k 20 --steps 4 --warmup 2 > $out/prof_k20.log 2>&1
echo rc=$?
