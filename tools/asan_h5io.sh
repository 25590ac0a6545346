#!/bin/bash
# Build csrc/h5ad/h5io.cpp with AddressSanitizer + UBSan (host code) and run the
# round-trip script through an embedding driver that links the sanitizer runtimes.
# usage: bash tools/asan_h5io.sh   (CPU only; no GPU involved)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
# builds are kept (build/ is neither in git nor sent to the GPU box) and redone only when
# a source is newer than its output: the compile was ~60 s of the CPU test suite
OUT=${CNMF_ASAN_DIR:-$ROOT/build/asan}
mkdir -p "$OUT"
EXT=$(python3 -c "import sysconfig; print(sysconfig.get_config_var('EXT_SUFFIX'))")
PYINC=$(python3 -c "import sysconfig, pybind11; print('-I' + sysconfig.get_paths()['include'] + ' -I' + pybind11.get_include())")
HDF5=${CNMF_HDF5_PREFIX:-/opt/conda}
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -fno-sanitize-recover=undefined -g -O1"
stale() {  # stale OUTPUT SOURCE...: the output is missing or older than a source
  local o=$1; shift
  [ -e "$o" ] || return 0
  for s_ in "$@"; do [ "$s_" -nt "$o" ] && return 0; done
  return 1
}
if stale "$OUT/_h5io$EXT" "$ROOT/csrc/h5ad/h5io.cpp" "$0"; then
  g++ -std=c++17 -shared -fPIC $SAN $PYINC -I"$HDF5/include" "$ROOT/csrc/h5ad/h5io.cpp" \
      "$HDF5/lib/libhdf5.so" -Wl,-rpath,/lib/x86_64-linux-gnu -Wl,-rpath,"$HDF5/lib" \
      -o "$OUT/_h5io$EXT"   # system sanitizer runtimes first: conda ships older ones
fi
if stale "$OUT/h5io_driver" "$ROOT/tools/asan/h5io_driver.cpp" "$0"; then
  g++ -std=c++17 -fno-pie $SAN $PYINC "$ROOT/tools/asan/h5io_driver.cpp" $(python3-config --ldflags --embed) \
      -no-pie -o "$OUT/h5io_driver"
fi
# the sanitizer runtime is linked into the driver executable; a pre-existing preload
# must not make ASan abort on link order
ASAN_OPTIONS=${ASAN_OPTIONS:-verify_asan_link_order=0:detect_leaks=0} \
UBSAN_OPTIONS=${UBSAN_OPTIONS:-print_stacktrace=1} \
PYTHONPATH="$(python3 -c 'import numpy, os; print(os.path.dirname(os.path.dirname(numpy.__file__)))')" \
    "$OUT/h5io_driver" "$OUT" "$ROOT/tools/asan/h5io_roundtrip.py"
