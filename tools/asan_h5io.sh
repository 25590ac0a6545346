#!/bin/bash
# Build csrc/h5ad/h5io.cpp with AddressSanitizer + UBSan (host code) and run the
# round-trip script through an embedding driver that links the sanitizer runtimes.
# usage: bash tools/asan_h5io.sh   (CPU only; no GPU involved)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/cnmf_asan
mkdir -p "$OUT"
EXT=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC=$(python3 -c "import sysconfig, pybind11; print('-I' + sysconfig.get_paths()['include'] + ' -I' + pybind11.get_include())")
HDF5=${CNMF_HDF5_PREFIX:-/opt/conda}
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g -O1"
g++ -std=c++17 -shared -fPIC $SAN $PYINC -I"$HDF5/include" "$ROOT/csrc/h5ad/h5io.cpp" \
    "$HDF5/lib/libhdf5.so" -Wl,-rpath,/lib/x86_64-linux-gnu -Wl,-rpath,"$HDF5/lib" \
    -o "$OUT/_h5io$EXT"   # system sanitizer runtimes first: conda ships older ones
g++ -std=c++17 -fno-pie $SAN $PYINC "$ROOT/tools/asan/h5io_driver.cpp" $(python3-config --ldflags --embed) \
    -no-pie -o "$OUT/h5io_driver"
# the sanitizer runtime is linked into the driver executable; a pre-existing preload
# must not make ASan abort on link order
ASAN_OPTIONS=${ASAN_OPTIONS:-verify_asan_link_order=0:detect_leaks=0} \
UBSAN_OPTIONS=${UBSAN_OPTIONS:-print_stacktrace=1} \
PYTHONPATH="$(python3 -c 'import numpy, os; print(os.path.dirname(os.path.dirname(numpy.__file__)))')" \
    "$OUT/h5io_driver" "$OUT" "$ROOT/tools/asan/h5io_roundtrip.py"
