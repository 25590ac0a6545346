"""In-tree native build for cnmf_torch_amd.

Builds two extension modules next to the Python sources so they travel with the
repository snapshot to the GPU box:

* ``cnmf_torch_amd/ops/_hip*.so`` -- every ``csrc/kernels/*.hip`` kernel plus the
  pybind11 bindings, compiled by ``hipcc --offload-arch=gfx950`` (CDNA4 only).
* ``cnmf_torch_amd/utils/_h5io*.so`` -- the native HDF5 layer used for h5ad I/O,
  compiled by the host C++ compiler against libhdf5.

Object files are cached under ``build/native`` and rebuilt when a source or any
header is newer.  Usage: ``python -m cnmf_torch_amd._build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
PKG = os.path.join(ROOT, "cnmf_torch_amd")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = "gfx950"       # MI355X (CDNA4) only

HIP_OUT = os.path.join(PKG, "ops", "_hip" + EXT)
H5_OUT = os.path.join(PKG, "utils", "_h5io" + EXT)
NPZ_OUT = os.path.join(PKG, "utils", "_npzio" + EXT)

HDF5_PREFIXES = [os.environ.get("CNMF_HDF5_PREFIX", ""), "/opt/conda", "/usr", "/usr/local"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC)")


def _py_includes() -> list[str]:
    import pybind11

    return ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"]]


def _headers() -> list[str]:
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _stale(out: str, deps: list[str]) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("command failed:\n  " + " ".join(cmd) + "\n" + r.stdout)


def build_hip(force: bool = False, jobs: int = 8, verbose: bool = True) -> str:
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    srcs.append(os.path.join(CSRC, "bindings.cpp"))
    hdrs = _headers()
    common = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-I" + CSRC,
              "-Wno-unused-result", "-munsafe-fp-atomics"]
    objs, todo = [], []
    # per-unit flags: the split-bf16 beta kernels keep their MFMA accumulators in VGPRs
    # (the elementwise work reads every accumulator: AGPR copies cost ~30 % of the VALU)
    # the pipelined solve keeps its elementwise update scalar: SLP-packed v_pk_*_f32 beside
    # MFMAs cost more issue cycles than the scalar pair (MI355X_MICROARCH.md cycle table)
    unit_flags = {os.path.basename(s): ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]
                  for s in srcs if os.path.basename(s).startswith("beta_planes")}
    # CNMF_PIPE_STAMPS_BUILD=1: the pipelined solve with its diagnostic phase stamps
    # (tools/pipe_stamp_probe.py); a changed flag set rebuilds the unit
    stamps = os.environ.get("CNMF_PIPE_STAMPS_BUILD", "0") == "1"
    for s in srcs:      # every instantiation unit of the pipelined solve (solve_pipe*.hip)
        if os.path.basename(s).startswith("solve_pipe"):
            unit_flags[os.path.basename(s)] = ["-fno-slp-vectorize"] + \
                (["-DCNMF_PIPE_STAMPS"] if stamps else [])
    for s in srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        flags_fn = o + ".flags"
        flags = " ".join(common + unit_flags.get(os.path.basename(s), []))
        old_flags = open(flags_fn).read() if os.path.exists(flags_fn) else None
        if force or old_flags != flags or _stale(o, [s] + hdrs):
            extra = _py_includes() if s.endswith(".cpp") else []
            todo.append(([hipcc, "-c", s, "-o", o] + common + extra +
                         unit_flags.get(os.path.basename(s), []), flags_fn, flags))
    if todo:
        if verbose:
            print(f"[cnmf build] compiling {len(todo)} HIP/C++ unit(s) for {ARCH}", flush=True)
        with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
            for f, (_, flags_fn, flags) in [(ex.submit(_run, c[0]), c) for c in todo]:
                f.result()
                with open(flags_fn, "w") as fh:      # recorded once the unit built
                    fh.write(flags)
    if force or todo or _stale(HIP_OUT, objs):
        tmp = HIP_OUT + ".tmp"
        _run([hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", tmp] + objs)
        os.replace(tmp, HIP_OUT)
        if verbose:
            print(f"[cnmf build] linked {os.path.relpath(HIP_OUT, ROOT)}", flush=True)
    return HIP_OUT


def _hdf5_prefix() -> str:
    for p in HDF5_PREFIXES:
        if p and os.path.exists(os.path.join(p, "include", "hdf5.h")) and glob.glob(
                os.path.join(p, "lib", "libhdf5.so*")):
            return p
    raise RuntimeError("libhdf5 headers/libs not found (set CNMF_HDF5_PREFIX)")


def build_h5(force: bool = False, verbose: bool = True) -> str:
    src = os.path.join(CSRC, "h5ad", "h5io.cpp")
    if not (force or _stale(H5_OUT, [src])):
        return H5_OUT
    prefix = _hdf5_prefix()
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    tmp = H5_OUT + ".tmp"
    cmd = [cxx, "-O2", "-shared", "-fPIC", "-std=c++17", "-pthread", src, "-o", tmp,
           "-I" + os.path.join(prefix, "include")] + _py_includes() + [
           "-L" + os.path.join(prefix, "lib"), "-lhdf5",
           "-Wl,-rpath," + os.path.join(prefix, "lib")]
    if verbose:
        print(f"[cnmf build] compiling native h5ad layer against {prefix}", flush=True)
    _run(cmd)
    os.replace(tmp, H5_OUT)
    return H5_OUT


def build_npz(force: bool = False, verbose: bool = True) -> str:
    """Native replicate-file writer (csrc/io/npzio.cpp): host C++, std::thread, zlib."""
    src = os.path.join(CSRC, "io", "npzio.cpp")
    if not (force or _stale(NPZ_OUT, [src])):
        return NPZ_OUT
    cxx = os.environ.get("CXX", shutil.which("g++") or "c++")
    tmp = NPZ_OUT + ".tmp"
    if verbose:
        print("[cnmf build] compiling native npz writer", flush=True)
    _run([cxx, "-O3", "-shared", "-fPIC", "-std=c++17", "-pthread", src, "-o", tmp]
         + _py_includes() + ["-lz"])
    os.replace(tmp, NPZ_OUT)
    return NPZ_OUT


def build_all(force: bool = False, jobs: int = 8, verbose: bool = True) -> list[str]:
    with cf.ThreadPoolExecutor(max_workers=3) as ex:
        fh = ex.submit(build_hip, force, jobs, verbose)
        f5 = ex.submit(build_h5, force, verbose)
        fn = ex.submit(build_npz, force, verbose)
        return [fh.result(), f5.result(), fn.result()]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--only", choices=["hip", "h5", "npz"], default=None)
    a = ap.parse_args(argv)
    if a.only == "hip":
        print(build_hip(a.force, a.jobs))
    elif a.only == "h5":
        print(build_h5(a.force))
    elif a.only == "npz":
        print(build_npz(a.force))
    else:
        for p in build_all(a.force, a.jobs):
            print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
