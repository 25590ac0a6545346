# PMC pass over the fused Lloyd step
export TMPDIR=/tmp
R=$(pwd)
out=$R/gpurun_out/r5s
mkdir -p $out
timeout -k 10 120 python tools/kmeans_probe.py > $out/probe.log 2>&1 && cat $out/probe.log &&
(cd /tmp && timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU -d $out/pmc -o km --output-format csv -- python $R/tools/kmeans_probe.py > $out/pmc.log 2>&1) && echo pmc_ok
echo rc=$?
