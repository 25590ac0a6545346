# mixed-K fused DP step (2 processes, cooperative slices) + xgmi tests
export TMPDIR=/tmp
out=gpurun_out/r5y
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" $out/pytest.log | tail -8; [ $rc -eq 0 ] || { grep -E "Error|assert" $out/pytest.log | head -20; exit 1; }
echo rc=$?
