# e2e x3: parallel prewarm groups + warmed figure child
export TMPDIR=/tmp
out=gpurun_out/r5zk
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1 || { echo E2E_FAILED; tail -20 $out/e2e$i.log; exit 1; }
  tail -n 1 $out/e2e$i.log | cut -c1-230
done
