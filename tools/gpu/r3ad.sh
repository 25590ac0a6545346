# norm counts streamed from the device into the h5ad: GPU test + Harmony 500k e2e (prepare stage) + PBMC e2e
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ad
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py tests/test_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 450 python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 --profile-stages $out/prof > $out/harmony.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
echo done
