# Compaction threshold A/B (0.75 vs 0.5, interleaved, 3 more pairs); KL fp16 counts default 'w' vs both vs off; KL GPU tests
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ak
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "kl or beta" > $out/pytest.log 2>&1
for i in 1 2 3; do
  for f in 0.5 0.75; do
    CNMF_COMPACT_FRAC_SMALL=$f timeout -k 10 120 python bench.py > $out/bench_cf${f}_$i.log 2>&1
  done
done
for i in 1 2; do
  for v in w 1 0; do
    CNMF_KL_FP16_COUNTS=$v timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl_${v}_$i.log 2>&1
  done
done
echo done
