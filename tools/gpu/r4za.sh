# XCD-map rule A/B: 75 % share (rule 1) vs whole budget on single-round launches (rule 2)
export TMPDIR=/tmp
out=gpurun_out/r4za
mkdir -p $out
for rep in 1 2; do
  for r in 2 1; do
    CNMF_PIPE_MAP_RULE=$r timeout -k 10 120 python bench.py > $out/bench_r${r}_$rep.log 2>&1 || exit 1
  done
done &&
for r in 2 1; do
  CNMF_PIPE_MAP_RULE=$r timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_r$r.log 2>&1 &&
  CNMF_PIPE_MAP_RULE=$r timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30_r$r.log 2>&1 &&
  CNMF_PIPE_MAP_RULE=$r timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_r$r.log 2>&1 || exit 1
done
echo rc=$?
