# KL engine on the split-bf16 kernels: GPU tests, probe, KL bench + kernel trace, Frobenius bench.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "split_bf16 or beta or nmf" > $out/pytest.log 2>&1
timeout -k 10 120 python tools/beta_probe2.py > $out/probe.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl -o run -- python3 bench.py --beta-loss kullback-leibler --steps 1 --warmup 1 > $out/prof_kl.log 2>&1
python tools/prof_summary.py $out/prof_kl/run_results.db --top 15 > $out/kl_kernels.txt 2>&1 || true
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
