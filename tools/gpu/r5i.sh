# Harmony stage: wall-clock, kernel summary, config-5 bench with cProfile and GPU-busy
export TMPDIR=/tmp
R=$(pwd)
out=$R/gpurun_out/r5i
mkdir -p $out
timeout -k 10 300 python tools/harmony_stage.py --repeat 2 > $out/stage.log 2>&1 && tail -n 1 $out/stage.log &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o hs -- python $R/tools/harmony_stage.py > $out/stage_prof.log 2>&1) && echo profiled &&
timeout -k 10 600 python tools/bench_harmony.py --profile $out/harmony_cprofile.txt --profile-stages $out/stage > $out/bench.log 2>&1 && tail -n 1 $out/bench.log &&
timeout -k 10 600 python tools/bench_harmony.py --gpu-busy > $out/bench_busy.log 2>&1 && tail -n 1 $out/bench_busy.log
echo rc=$?
