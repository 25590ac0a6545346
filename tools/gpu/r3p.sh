# e2e with figure prestart + native PNG writer + concurrent k-selection; fused raw-slab cap A/B
set -e
export TMPDIR=/tmp
out=gpurun_out/r3p
mkdir -p $out
for i in 1 2; do timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1; done
timeout -k 10 120 python bench.py > $out/bench_s4.log 2>&1
CNMF_FUSED_MAX_SLABS=16 timeout -k 10 120 python bench.py > $out/bench_s16.log 2>&1
CNMF_FUSED_MAX_SLABS=8 timeout -k 10 120 python bench.py > $out/bench_s8.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_s4b.log 2>&1
CNMF_FUSED_MAX_SLABS=16 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/grid_s16.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 10 --warmup 3 > $out/grid_s4.log 2>&1
echo done
