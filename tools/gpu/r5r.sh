# k-means counting sort; emulated-world projection at the measured latency
export TMPDIR=/tmp
R=$(pwd)
out=$R/gpurun_out/r5r
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_preprocess.py -x -v --timeout 170 --timeout-method thread -k "kmeans or harmony" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -n 1 $out/pytest.log
timeout -k 10 300 python tools/harmony_stage.py --repeat 2 > $out/stage.log 2>&1 && tail -n 1 $out/stage.log | cut -c1-120 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o hs -- python $R/tools/harmony_stage.py > $out/stage_prof.log 2>&1) && echo profiled &&
echo rc=$?
echo rc=$?
