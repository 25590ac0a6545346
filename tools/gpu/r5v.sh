# full GPU suite after the nmf split + KL baselines (dense, CSR 8 %)
export TMPDIR=/tmp
out=gpurun_out/r5v
mkdir -p $out
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?; tail -n 2 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head -20; exit 1; }
timeout -k 10 300 python bench.py > $out/bench.log 2>&1 && tail -n 1 $out/bench.log | cut -c1-160 &&
timeout -k 10 300 python bench.py --beta-loss kullback-leibler --steps 5 --warmup 1 > $out/kl.log 2>&1 && tail -n 1 $out/kl.log | cut -c1-160 &&
timeout -k 10 300 python bench.py --beta-loss kullback-leibler --density 0.08 --steps 5 --warmup 1 > $out/kl08.log 2>&1 && tail -n 1 $out/kl08.log | cut -c1-160 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof08 -o kl -- python $GRAFT_REPO_ROOT/bench.py --beta-loss kullback-leibler --density 0.08 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$out/kl08prof.log 2>&1) && echo profiled
echo rc=$?
