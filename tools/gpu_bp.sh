# split-bf16 beta kernels: GPU tests + probe timings.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "split_bf16 or beta" > $out/pytest.log 2>&1
timeout -k 10 120 python tools/beta_probe2.py > $out/probe.log 2>&1
