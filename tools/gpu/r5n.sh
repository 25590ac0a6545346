# K=17..20 eight-tile usage solve (one co-resident round at 100 x 5000) + k-means phase B
export TMPDIR=/tmp
R=$(pwd)
out=$R/gpurun_out/r5n
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_solve_pipe_gpu.py tests/test_preprocess.py -x -v --timeout 170 --timeout-method thread -k "kmeans or harmony or pipe or wide or fused_online" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -n 1 $out/pytest.log
timeout -k 10 300 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20a.log 2>&1 && tail -n 1 $out/k20a.log | cut -c1-160 &&
timeout -k 10 300 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20b.log 2>&1 && tail -n 1 $out/k20b.log | cut -c1-160 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof20 -o k20 -- python $R/bench.py --k 20 --steps 3 --warmup 1 > $out/k20prof.log 2>&1) && echo profiled20 &&
timeout -k 10 300 python tools/harmony_stage.py --repeat 2 > $out/stage.log 2>&1 && tail -n 1 $out/stage.log | cut -c1-120 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o hs -- python $R/tools/harmony_stage.py > $out/stage_prof.log 2>&1) && echo profiled
echo rc=$?
