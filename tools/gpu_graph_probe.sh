# eager vs HIP-graph pass replay probe
# usage: bash tools/gpu_graph_probe.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 200 python -u tools/graph_probe.py > $out/graph_probe.log 2>&1
