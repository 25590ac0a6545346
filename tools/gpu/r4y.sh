# sparse KL: LDS-variant workgroup width A/B (staging traffic vs parallelism)
export TMPDIR=/tmp
out=gpurun_out/r4y
mkdir -p $out
for d in 0.08 0.15; do
  for c in 128 256 512 64; do
    CNMF_KL_COLS=$c timeout -k 10 200 python bench.py --beta-loss kullback-leibler --density $d --steps 3 --warmup 1 > $out/kl_${d}_c$c.log 2>&1 || exit 1
  done
done
echo rc=$?
