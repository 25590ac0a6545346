# e2e pipeline bench twice + Harmony config
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e1.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py --profile $out/e2e_cprofile.txt > $out/e2e2.log 2>&1
timeout -k 10 400 python tools/bench_harmony.py > $out/harmony.log 2>&1
