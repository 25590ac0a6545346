# stamps probe build: phase breakdown at K=10 / 20 after the prologue changes
export TMPDIR=/tmp
out=gpurun_out/r4o
mkdir -p $out
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 10 > $out/stamps_k10.log 2>&1 &&
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 20 > $out/stamps_k20.log 2>&1 &&
timeout -k 10 200 python tools/pipe_stamp_probe.py --k 30 > $out/stamps_k30.log 2>&1
echo rc=$?
