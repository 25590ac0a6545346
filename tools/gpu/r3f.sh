# e2e pipeline (+cProfile), new kernel tests (seg median, 2 B planes, GPU-vs-CPU tolerance),
# float-input bench, 10M x 5k planes-only on one GPU.
set -e
export TMPDIR=/tmp
out=gpurun_out/r3f
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "seg_median or two_b_planes or gpu_matches_cpu or cluster_medians or fused or graph" > $out/pytest.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_cprofile.txt > $out/e2e_prof.log 2>&1
timeout -k 10 120 python bench.py --float-input > $out/bench_float.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 400 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 8 --planes-only > $out/large_10M_planes.log 2>&1
echo done
