# e2e x3: prewarm + figure prestart + X planes built ahead in prepare
export TMPDIR=/tmp
out=gpurun_out/r5zf
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1 || { echo E2E_FAILED; tail -20 $out/e2e$i.log; exit 1; }
  tail -n 1 $out/e2e$i.log | cut -c1-260
done
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 170 --timeout-method thread -k "pipeline or consensus or e2e or kselect or k_selection or prewarm" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -n 1 $out/pytest.log
