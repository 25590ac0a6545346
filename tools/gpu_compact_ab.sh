# Compaction threshold / bucket A/B on the headline bench (same box).
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for cfg in "0.25 8" "0.125 8" "0.5 8" "0.25 4" "0.25 16" "0.25 8"; do
  set -- $cfg
  CNMF_COMPACT_FRAC=$1 CNMF_COMPACT_BUCKET=$2 timeout -k 10 120 python bench.py > $out/bench_f$1_b$2.log 2>&1
  echo "frac $1 bucket $2 $(tail -1 $out/bench_f$1_b$2.log | cut -c1-110)" >> $out/summary.txt
done
