set -e
export TMPDIR=/tmp
mkdir -p gpurun_out/r2p
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "solve or gemm or concurrent or graph" > gpurun_out/r2p/pytest.log 2>&1 || true
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r2p/counters.txt 2>&1 || true
for v in reg mfma; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/r2p/pmc1_$v -o run --output-format csv -- python3 tools/solve_pmc_probe.py $v > gpurun_out/r2p/pmc1_$v.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE -d gpurun_out/r2p/pmc2_$v -o run --output-format csv -- python3 tools/solve_pmc_probe.py $v > gpurun_out/r2p/pmc2_$v.log 2>&1 || true
done
