# Session restart: full GPU suite, smoke, headline/KL (fp16 counts on/w/off)/grid benches, KL kernel summary
set -e
export TMPDIR=/tmp
out=gpurun_out/r3v
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
for v in 1 w 0; do CNMF_KL_FP16_COUNTS=$v timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_$v.log 2>&1; done
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof_kl -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --steps 2 --warmup 1 > $out/prof_kl.log 2>&1
echo done
