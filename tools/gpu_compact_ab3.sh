# Size-dependent compaction threshold: NMF GPU tests, headline 3x and K-grid 2x (same box).
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 150 --timeout-method thread -k "nmf or grid or ragged or early or graph" > $out/pytest.log 2>&1
for i in 1 2 3; do
  timeout -k 10 120 python bench.py > $out/b$i.log 2>&1
  echo "headline $(tail -1 $out/b$i.log | cut -c60-100)" >> $out/summary.txt
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/g$i.log 2>&1
  echo "grid $(tail -1 $out/g$i.log | cut -c60-110)" >> $out/summary.txt
done
CNMF_COMPACT_FRAC_SMALL=0.25 timeout -k 10 120 python bench.py > $out/b_old.log 2>&1
echo "headline old-rule $(tail -1 $out/b_old.log | cut -c60-100)" >> $out/summary.txt
