# pipelined MU sweep: per-tile eps check (min3 + one compare) instead of per-element select
export TMPDIR=/tmp
out=gpurun_out/r5zc
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 170 --timeout-method thread -k "solve or fused or pipe" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -n 1 $out/pytest.log
timeout -k 10 300 python bench.py > $out/b1.log 2>&1 && tail -n 1 $out/b1.log | cut -c1-140 &&
timeout -k 10 300 python bench.py > $out/b2.log 2>&1 && tail -n 1 $out/b2.log | cut -c1-140 &&
timeout -k 10 300 python bench.py --k 20 > $out/k20.log 2>&1 && tail -n 1 $out/k20.log | cut -c1-140 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/profh -o h -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$out/hprof.log 2>&1) && echo profiled_headline
echo rc=$?
