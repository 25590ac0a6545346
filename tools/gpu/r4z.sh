# XCD-map threshold A/B (share of the per-XCD resident budget)
export TMPDIR=/tmp
out=gpurun_out/r4z
mkdir -p $out
for pct in 75 100 50; do
  CNMF_PIPE_MAP_PCT=$pct timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_p$pct.log 2>&1 &&
  CNMF_PIPE_MAP_PCT=$pct timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30_p$pct.log 2>&1 &&
  CNMF_PIPE_MAP_PCT=$pct timeout -k 10 120 python bench.py > $out/bench_p$pct.log 2>&1 || exit 1
done
echo rc=$?
