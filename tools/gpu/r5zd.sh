# solve phase breakdown at HEAD (stamped probe build): K=10 at the stream's 137 live slots and 100, K=20
export TMPDIR=/tmp
out=gpurun_out/r5zd
mkdir -p $out
timeout -k 10 300 python tools/pipe_stamp_probe.py --k 10 --reps 137 > $out/k10_137.log 2>&1 && tail -n 4 $out/k10_137.log | cut -c1-400 &&
timeout -k 10 300 python tools/pipe_stamp_probe.py --k 10 --reps 100 > $out/k10_100.log 2>&1 && tail -n 4 $out/k10_100.log | cut -c1-400 &&
timeout -k 10 300 python tools/pipe_stamp_probe.py --k 20 --reps 100 > $out/k20.log 2>&1 && tail -n 4 $out/k20.log | cut -c1-400
echo rc=$?
