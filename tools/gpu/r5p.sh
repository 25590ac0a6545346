# packed DP step + one-shot xGMI RS/AG kernels; k-means tiles; emulated-world projection
export TMPDIR=/tmp
R=$(pwd)
out=$R/gpurun_out/r5p
mkdir -p $out
true

true &&

timeout -k 10 400 python tools/bench_large.py --cells 1000000 --genes 2000 --k 10 --reps 100 --dp --emulate-world 8 --steps 2 --warmup 1 > $out/emu8_1m.log 2>&1 && tail -n 1 $out/emu8_1m.log &&
timeout -k 10 500 python tools/bench_large.py --cells 10000000 --genes 5000 --k 20 --reps 25 --dp --emulate-world 8 --planes-only --steps 1 > $out/emu8_10m.log 2>&1 && tail -n 1 $out/emu8_10m.log &&
timeout -k 10 300 python tools/harmony_stage.py --repeat 2 > $out/stage.log 2>&1 && tail -n 1 $out/stage.log | cut -c1-120 &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o hs -- python $R/tools/harmony_stage.py > $out/stage_prof.log 2>&1) && echo profiled
echo rc=$?
