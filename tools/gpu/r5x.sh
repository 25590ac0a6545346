# K=20: batch vs stream schedule; GEMM plan sweep at M = 2000
export TMPDIR=/tmp
out=gpurun_out/r5x
mkdir -p $out
timeout -k 10 300 python bench.py --k 20 --schedule batch --steps 5 --warmup 2 > $out/k20b.log 2>&1 && tail -n 1 $out/k20b.log | cut -c1-140 &&
timeout -k 10 300 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20s.log 2>&1 && tail -n 1 $out/k20s.log | cut -c1-140 &&
timeout -k 10 300 python tools/gemm_plan_sweep.py 2000 1500 > $out/sweep.log 2>&1 && cut -c1-2000 $out/sweep.log &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof -o k -- python $GRAFT_REPO_ROOT/bench.py --k 20 --schedule batch --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/$out/prof.log 2>&1) && echo profiled
echo rc=$?
