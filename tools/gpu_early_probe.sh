# factorize with / without early replicate writes, alternating in one process
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u tools/early_write_probe.py > $out/probe.log 2>&1
