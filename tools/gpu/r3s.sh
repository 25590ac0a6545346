# tail passes: cap the fused GEMM's k split at the raw-slab limit (no gemm_reduce) A/B
set -e
export TMPDIR=/tmp
out=gpurun_out/r3s
mkdir -p $out
timeout -k 10 120 python bench.py > $out/bench_a.log 2>&1
CNMF_FUSED_CAP_KSPLIT=1 timeout -k 10 120 python bench.py > $out/bench_cap.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_b.log 2>&1
CNMF_FUSED_CAP_KSPLIT=1 timeout -k 10 120 python bench.py > $out/bench_cap2.log 2>&1
CNMF_FUSED_CAP_KSPLIT=1 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/grid_cap.log 2>&1
CNMF_FUSED_CAP_KSPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/prof.log 2>&1
echo done
