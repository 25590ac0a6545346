# headline: host cProfile of steady-state steps + kernel trace per pass (last 2 runs)
set -e
export TMPDIR=/tmp
out=gpurun_out/r3r
mkdir -p $out
timeout -k 10 200 python tools/step_cprofile.py frobenius 10 > $out/step_cprofile.txt 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/prof.log 2>&1
echo done
