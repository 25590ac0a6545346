# Host-path check: NMF/solve GPU tests, bench 3x, host cProfile of bench steps, graph probe.
# usage: bash tools/gpu_host.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "nmf or solve or graph or grid or ragged" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench1.log 2>&1
timeout -k 10 120 python bench.py > $out/bench2.log 2>&1
timeout -k 10 120 python bench.py > $out/bench3.log 2>&1
timeout -k 10 200 python -u tools/graph_probe.py > $out/graph_probe.log 2>&1
timeout -k 10 200 python -u tools/step_cprofile.py frobenius 10 > $out/cprofile.log 2>&1
