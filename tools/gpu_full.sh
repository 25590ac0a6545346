# Full GPU validation: every gpu test, smoke, bench (Frobenius + KL).
# usage: bash tools/gpu_full.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
