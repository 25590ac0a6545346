set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_xgmi_gpu.py -x -v --timeout 150 --timeout-method thread > $out/pytest_xgmi.log 2>&1
