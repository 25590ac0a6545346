# prewarm: serial vs one thread per group (fresh processes), then e2e x3
export TMPDIR=/tmp
out=gpurun_out/r5zj
mkdir -p $out
for m in "--serial" "" "--serial" ""; do
  timeout -k 10 120 python tools/prewarm_probe.py $m 2>&1 | grep prewarm_s
done
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1 || { echo E2E_FAILED; tail -20 $out/e2e$i.log; exit 1; }
  tail -n 1 $out/e2e$i.log | cut -c1-230
done
timeout -k 10 300 python -u -m pytest tests/test_prewarm.py -m gpu -x -v --timeout 170 --timeout-method thread > $out/pytest.log 2>&1; tail -n 1 $out/pytest.log
