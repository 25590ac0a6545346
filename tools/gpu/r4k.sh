# e2e with cProfile, float-input bench, KL at 0.08 (standard config), K=10 grid
export TMPDIR=/tmp
out=gpurun_out/r4k
mkdir -p $out
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1 &&
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_prof.txt > $out/e2e_prof.log 2>&1 &&
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density 0.08 --steps 3 --warmup 1 > $out/kl_d08.log 2>&1 &&
timeout -k 10 200 python bench.py --float-input --steps 10 --warmup 3 > $out/float.log 2>&1 &&
timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
echo rc=$?
CNMF_FUSED_MAX_SLABS=8 timeout -k 10 120 python bench.py > gpurun_out/r4k/bench_slabs8.log 2>&1 &&
timeout -k 10 120 python bench.py > gpurun_out/r4k/bench_slabs4.log 2>&1
echo rc2=$?
CNMF_PIPE_BALANCE=1 timeout -k 10 120 python bench.py > gpurun_out/r4k/bench_bal.log 2>&1 &&
CNMF_PIPE_BALANCE=1 timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > gpurun_out/r4k/k20_bal.log 2>&1 &&
timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > gpurun_out/r4k/k20.log 2>&1 &&
CNMF_PIPE_BALANCE=1 timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > gpurun_out/r4k/k30_bal.log 2>&1 &&
timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > gpurun_out/r4k/k30.log 2>&1
echo rc3=$?
CNMF_GEMM_KSPLIT=2 timeout -k 10 120 python bench.py > gpurun_out/r4k/bench_ks2.log 2>&1 &&
CNMF_GEMM_KSPLIT=1 timeout -k 10 120 python bench.py > gpurun_out/r4k/bench_ks1.log 2>&1
echo rc4=$?
