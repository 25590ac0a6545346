# k-means counting sort; emulated-world projection at the measured latency
export TMPDIR=/tmp
R=$(pwd)
out=$R/gpurun_out/r5q
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_preprocess.py -x -v --timeout 170 --timeout-method thread -k "kmeans or harmony" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -n 1 $out/pytest.log
timeout -k 10 300 python tools/harmony_stage.py --repeat 2 > $out/stage.log 2>&1 && tail -n 1 $out/stage.log | cut -c1-120 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o hs -- python $R/tools/harmony_stage.py > $out/stage_prof.log 2>&1) && echo profiled &&
timeout -k 10 400 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --dp --emulate-world 8 --steps 2 --warmup 1 > $out/emu8_1m.log 2>&1 && tail -n 1 $out/emu8_1m.log | cut -c 1-200 &&
timeout -k 10 500 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 25 --dp --emulate-world 8 --planes-only --steps 1 > $out/emu8_10m.log 2>&1 && tail -n 1 $out/emu8_10m.log | cut -c 1-200
echo rc=$?
