# e2e x4 (planes ahead + prewarm), the last one with cProfile
export TMPDIR=/tmp
out=gpurun_out/r5zi
mkdir -p $out
for i in 1 2 3; do
  timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1 || { echo E2E_FAILED; tail -20 $out/e2e$i.log; exit 1; }
  tail -n 1 $out/e2e$i.log | cut -c1-230
done
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_cprofile.txt > $out/e2e4.log 2>&1 && tail -n 1 $out/e2e4.log | cut -c1-230
