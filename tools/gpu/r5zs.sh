# e2e x4 with cProfile per stage: catch the factorize outliers
export TMPDIR=/tmp
out=gpurun_out/r5zs
mkdir -p $out
for i in 1 2 3 4; do
  timeout -k 10 300 python tools/bench_e2e.py --profile $out/prof$i.txt > $out/e2e$i.log 2>&1 || { echo E2E_FAILED; tail -20 $out/e2e$i.log; exit 1; }
  tail -n 1 $out/e2e$i.log | cut -c1-160
done
