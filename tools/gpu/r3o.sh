# full GPU suite after the KL work; e2e with concurrent k-selection; headline bench
set -e
export TMPDIR=/tmp
out=gpurun_out/r3o
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e2.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
echo done
