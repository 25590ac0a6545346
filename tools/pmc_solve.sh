# PMC passes of the fused solve (tools/solve_pmc_probe.py: sweeps only, no mid-solve
# objective checks) for the VALU-resident and matrix-core variants.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
for v in reg mfma; do
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $out/kt_$v -o run --output-format csv -- python3 tools/solve_pmc_probe.py $v 1000 > $out/kt_$v.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d $out/pmc1_$v -o run --output-format csv -- python3 tools/solve_pmc_probe.py $v 1000 > $out/pmc1_$v.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $out/pmc2_$v -o run --output-format csv -- python3 tools/solve_pmc_probe.py $v 1000 > $out/pmc2_$v.log 2>&1
done
