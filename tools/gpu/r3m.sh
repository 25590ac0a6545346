# KL kernel bound probe: X traffic removed (CNMF_BP_XPROBE) vs normal, CT 1 / 2
set -e
export TMPDIR=/tmp
out=gpurun_out/r3m
mkdir -p $out
for ct in 2 1; do
CNMF_BP_KL_CT=$ct timeout -k 10 120 python tools/beta_probe2.py > $out/probe_ct$ct.log 2>&1
CNMF_BP_KL_CT=$ct CNMF_BP_XPROBE=1 timeout -k 10 120 python tools/beta_probe2.py > $out/probe_ct${ct}_noX.log 2>&1
done
echo done
