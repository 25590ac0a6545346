# host pass overheads A/B on one box: first pass of a recurring layout from its graph
# (CNMF_LAYOUT_REPLAY) and the flag copy on a side stream (CNMF_FLAG_STREAM)
set -e
export TMPDIR=/tmp
out=gpurun_out/r3y
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused or graph or mixed_k or nmf_batch_gpu or concurrent or split_gemm" > $out/pytest.log 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py > $out/bench_on_$i.log 2>&1
  CNMF_LAYOUT_REPLAY=0 CNMF_FLAG_STREAM=0 timeout -k 10 120 python bench.py > $out/bench_off_$i.log 2>&1
  CNMF_FLAG_STREAM=0 timeout -k 10 120 python bench.py > $out/bench_replay_$i.log 2>&1
  CNMF_LAYOUT_REPLAY=0 timeout -k 10 120 python bench.py > $out/bench_stream_$i.log 2>&1
done
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_on.log 2>&1
CNMF_LAYOUT_REPLAY=0 CNMF_FLAG_STREAM=0 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_off.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/prof.log 2>&1
echo done
