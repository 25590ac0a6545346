# sparse KL: CSR entries cached across MU steps
export TMPDIR=/tmp
out=gpurun_out/r5w
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 170 --timeout-method thread -k "kl or sparse" > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; grep -E "Error|assert|FAILED|passed|failed" $out/pytest.log | head -30; exit 1; }
tail -n 1 $out/pytest.log
timeout -k 10 300 python bench.py --beta-loss kullback-leibler --density 0.08 --steps 5 --warmup 1 > $out/kl08.log 2>&1 && tail -n 1 $out/kl08.log | cut -c1-160 &&
timeout -k 10 300 python bench.py --beta-loss kullback-leibler --density 0.15 --steps 5 --warmup 1 > $out/kl15.log 2>&1 && tail -n 1 $out/kl15.log | cut -c1-160 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/prof08 -o kl -- python $GRAFT_REPO_ROOT/bench.py --beta-loss kullback-leibler --density 0.08 --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/$out/kl08prof.log 2>&1) && echo profiled
echo rc=$?
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$out/profh -o h -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$out/hprof.log 2>&1) && echo profiled_headline &&
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $GRAFT_REPO_ROOT/$out/pmckl -o kl --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --beta-loss kullback-leibler --density 0.08 --steps 1 --warmup 0 > $GRAFT_REPO_ROOT/$out/pmckl.log 2>&1) && echo pmc_kl
echo rc2=$?
