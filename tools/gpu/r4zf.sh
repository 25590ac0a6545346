# derived MfmaUtil / VALUBusy per kernel of one headline (K=10) and one K=20 step at HEAD
export TMPDIR=/tmp
out=gpurun_out/r4zf
mkdir -p $out
timeout -s KILL 120 rocprofv3 --pmc MfmaUtil --output-format csv -d $out/k10_MfmaUtil -o run -- python3 bench.py --steps 1 --warmup 1 > $out/k10_MfmaUtil.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc VALUBusy --output-format csv -d $out/k10_VALUBusy -o run -- python3 bench.py --steps 1 --warmup 1 > $out/k10_VALUBusy.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc MfmaUtil --output-format csv -d $out/k20_MfmaUtil -o run -- python3 bench.py --k 20 --steps 1 --warmup 1 > $out/k20_MfmaUtil.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc VALUBusy --output-format csv -d $out/k20_VALUBusy -o run -- python3 bench.py --k 20 --steps 1 --warmup 1 > $out/k20_VALUBusy.log 2>&1
echo rc=$?
