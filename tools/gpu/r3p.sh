# e2e with figure prestart + native PNG writer + concurrent k-selection
set -e
export TMPDIR=/tmp
out=gpurun_out/r3p
mkdir -p $out
for i in 1 2 3; do timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1; done
echo done
