# Early replicate writes: GPU pipeline test, e2e pipeline with and without, bench.
# usage: bash tools/gpu_early.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -x -v --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
CNMF_EARLY_WRITE=0 timeout -k 10 300 python tools/bench_e2e.py > $out/e2e_off.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e_on.log 2>&1
CNMF_EARLY_WRITE=0 timeout -k 10 300 python tools/bench_e2e.py > $out/e2e_off2.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e_on2.log 2>&1
