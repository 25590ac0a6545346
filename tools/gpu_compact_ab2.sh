# Compaction threshold A/B, repeated, headline + K-grid bench (same box).
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for f in 0.25 0.5 0.75 0.25 0.5 0.75; do
  CNMF_COMPACT_FRAC=$f timeout -k 10 120 python bench.py > $out/b.log 2>&1
  echo "frac $f $(tail -1 $out/b.log | cut -c60-100)" >> $out/summary.txt
done
for f in 0.25 0.5 0.25 0.5; do
  CNMF_COMPACT_FRAC=$f timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/g.log 2>&1
  echo "grid frac $f $(tail -1 $out/g.log | cut -c60-110)" >> $out/summary.txt
done
