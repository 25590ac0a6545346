# Short GPU pass: solve/GEMM tests, solve probe, bench, e2e pipeline bench.
# usage: bash tools/gpu_check2.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "solve or gemm or concurrent or graph or refit or coop or nmf" > $out/pytest.log 2>&1 || true
timeout -k 10 200 python -u tools/solve_probe.py > $out/solve.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_cprofile.txt > $out/e2e.log 2>&1
