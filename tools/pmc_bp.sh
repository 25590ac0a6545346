# PMC passes of the split-bf16 beta kernels (tools/bp_pmc_probe.py h|w).
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for v in h w; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/pmc1_$v -o run --output-format csv -- python3 tools/bp_pmc_probe.py $v > $out/pmc1_$v.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d $out/pmc2_$v -o run --output-format csv -- python3 tools/bp_pmc_probe.py $v > $out/pmc2_$v.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum -d $out/pmc3_$v -o run --output-format csv -- python3 tools/bp_pmc_probe.py $v > $out/pmc3_$v.log 2>&1
done
