# validation of the K-dependent slice width: full GPU suite, smoke, K=10 / 20 / 30 benches
export TMPDIR=/tmp
out=gpurun_out/r4zj
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 &&
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 150 python bench.py --k 20 > $out/k20.log 2>&1 &&
timeout -k 10 150 python bench.py --k 30 > $out/k30.log 2>&1 &&
timeout -k 10 150 python bench.py --k 20 > $out/k20b.log 2>&1
echo rc=$?
