# K=20 and K=30: continuous batching vs one batch per step (2 runs each, alternating)
export TMPDIR=/tmp
out=gpurun_out/r5zp
mkdir -p $out
for k in 20 30; do
  for s in stream batch stream batch; do
    timeout -k 10 300 python bench.py --k $k --schedule $s > $out/k${k}_$s.log 2>&1 || { echo FAILED; tail -5 $out/k${k}_$s.log; exit 1; }
    echo "k=$k $s $(tail -n 1 $out/k${k}_$s.log | cut -c1-110)"
  done
done
