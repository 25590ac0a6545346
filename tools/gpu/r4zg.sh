# final validation after the spawn-retry change in the test harness: xGMI tests, full GPU suite, smoke, headline
export TMPDIR=/tmp
out=gpurun_out/r4zg
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 170 --timeout-method thread > $out/pytest_xgmi.log 2>&1 && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest_xgmi.log $out/pytest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
echo rc=$?
