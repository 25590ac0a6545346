# One GPU validation pass: solve/GEMM kernel tests, solve probe, bench (default and with
# the VALU solve / exact 3-plane GEMMs for A/B), kernel-trace profile of bench.py.
# usage: bash tools/gpu_check.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "solve or gemm or concurrent or graph or refit or coop or nmf" > $out/pytest.log 2>&1 || true
timeout -k 10 200 python -u tools/solve_probe.py > $out/solve.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
CNMF_SOLVE_MFMA=0 timeout -k 10 120 python bench.py > $out/bench_nomfma.log 2>&1
CNMF_GEMM_APLANES=3 timeout -k 10 120 python bench.py > $out/bench_3planes.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
