# DP fused step: async exchanges per unit (K groups); single-K stays one unit
export TMPDIR=/tmp
out=gpurun_out/r5z
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" $out/pytest.log | tail -10; [ $rc -eq 0 ] || { grep -E "Error|assert" $out/pytest.log | head -20; exit 1; }
timeout -k 10 400 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --dp --emulate-world 8 --steps 2 --warmup 1 > $out/emu8_1m.log 2>&1 && tail -n 1 $out/emu8_1m.log | cut -c 1-200
echo rc=$?
