# compaction threshold A/B now that a compacted layout's first pass replays its graph
set -e
export TMPDIR=/tmp
out=gpurun_out/r3aj
mkdir -p $out
for i in 1 2; do
  for f in 0.75 0.5 0.6; do
    CNMF_COMPACT_FRAC_SMALL=$f timeout -k 10 120 python bench.py > $out/bench_cf${f}_$i.log 2>&1
  done
done
CNMF_COMPACT_FRAC_SMALL=0.5 timeout -k 10 200 rocprofv3 --kernel-trace -d $out/prof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/prof.log 2>&1
echo done
