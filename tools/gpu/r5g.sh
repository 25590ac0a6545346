# full GPU suite + smoke + headline after the streaming / slot-removal changes
export TMPDIR=/tmp
out=gpurun_out/r5g
mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log &&
timeout -k 10 200 python bench.py > $out/bench.log 2>&1 && tail -n 1 $out/bench.log | cut -c1-300
echo rc=$?
