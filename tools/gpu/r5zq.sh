# bench default schedule: K=20 / 30 one batch per step, K=10 stream
export TMPDIR=/tmp
out=gpurun_out/r5zq
mkdir -p $out
for a in "--k 20" "--k 20" "--k 30" ""; do
  n=$(echo "k${a}" | tr -d ' -')
  timeout -k 10 300 python bench.py $a > $out/$n.log 2>&1 || { echo FAILED; tail -5 $out/$n.log; exit 1; }
  echo "$a $(tail -n 1 $out/$n.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["config"]["schedule"][:60])')"
done
timeout -k 10 600 python -u -m pytest tests/test_bench_contract.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -n 1 $out/pytest.log; exit $rc
