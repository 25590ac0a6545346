# kernel traces of the Frobenius and KL benches for the idle-gap analysis
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace -d $out/prof_frob -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof_frob.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof_kl -o run -- python3 bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/prof_kl.log 2>&1
python tools/gap_summary.py $out/prof_frob/run_results.db --from-frac 0.5 --top 12 > $out/gaps_frob.txt 2>&1 || true
python tools/gap_summary.py $out/prof_kl/run_results.db --from-frac 0.4 --top 12 > $out/gaps_kl.txt 2>&1 || true
