# Round-end validation: every GPU test, smoke, Frobenius/KL bench, K-grid bench, e2e
# pipeline, kernel-trace profile.  usage: bash tools/gpu/round_end.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
timeout -k 10 300 python tools/bench_e2e.py > $out/e2e.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
