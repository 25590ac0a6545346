# Harmony long-reduction products as chunked batched GEMMs: tests, 500k e2e + kernel trace
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ae
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "harmony or preprocess" > $out/pytest.log 2>&1
timeout -k 10 450 python tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony.log 2>&1
timeout -k 10 450 rocprofv3 --kernel-trace --stats -d $out/prof_harmony -o run --output-format csv -- python3 tools/bench_harmony.py --cells 500000 --genes 3000 --hvg 2000 > $out/harmony_prof.log 2>&1
echo done
