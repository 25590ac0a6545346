# Host-side gap between bench steps: sync sites, torch.profiler attribution; bench after packing the coop flags into finalize's copy
set -e
export TMPDIR=/tmp
out=gpurun_out/r3al
mkdir -p $out
timeout -k 10 240 python -u tools/step_gap_probe.py > $out/gap.log 2>&1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "coop or nmf" > $out/pytest.log 2>&1
for i in 1 2 3; do timeout -k 10 120 python bench.py > $out/bench_$i.log 2>&1; done
echo done
