# ridge / exact-stats / harmony / e2e / DP emulation / GEMM ceiling / KL density
export TMPDIR=/tmp
out=gpurun_out/r4c
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_preprocess.py tests/test_pipeline_gpu.py -k "ridge or exact or moe or harmony or dense or streamed or pipe" -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 10 > $out/stamps_k10.log 2>&1 &&
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 20 > $out/stamps_k20.log 2>&1 &&
timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20.log 2>&1 &&
timeout -k 10 200 python tools/gemm_ceiling_probe.py > $out/gemm_ceiling.log 2>&1 &&
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1 &&
timeout -k 10 300 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --dp --emulate-world 8 --steps 2 --warmup 1 > $out/emu8_1m.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_emu8_1m -o run --output-format csv -- python3 tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --dp --emulate-world 8 --steps 1 > $out/prof_emu8_1m.log 2>&1 &&
timeout -k 10 400 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 25 --dp --emulate-world 8 --planes-only --steps 1 > $out/emu8_10m.log 2>&1 &&
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density 0.08 --steps 3 --warmup 1 > $out/kl_d08_sparse.log 2>&1 &&
CNMF_KL_SPARSE=0 timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density 0.08 --steps 3 --warmup 1 > $out/kl_d08_dense.log 2>&1 &&
timeout -k 10 600 python tools/bench_harmony.py > $out/harmony.log 2>&1
echo rc=$?
