# full GPU suite + headline bench x2 + KL/K20 benches
export TMPDIR=/tmp
out=gpurun_out/r5t
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -n 3 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit 1; }
timeout -k 10 300 python bench.py > $out/bench1.log 2>&1 && tail -n 1 $out/bench1.log | cut -c1-200 &&
timeout -k 10 300 python bench.py > $out/bench2.log 2>&1 && tail -n 1 $out/bench2.log | cut -c1-200 &&
timeout -k 10 300 python bench.py --kmin 5 --kmax 13 > $out/grid.log 2>&1 && tail -n 1 $out/grid.log | cut -c1-200
echo rc=$?
