# e2e pipeline x3 + cProfile
export TMPDIR=/tmp
out=gpurun_out/r5u
mkdir -p $out
for i in 1 2 3; do timeout -k 10 300 python tools/bench_e2e.py > $out/e2e$i.log 2>&1 || exit 1; tail -n 1 $out/e2e$i.log | cut -c1-400; done
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_cprofile.txt > $out/e2e_prof.log 2>&1 && echo profiled
echo rc=$?
