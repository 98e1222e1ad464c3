"""In-tree builder of the native extensions (no hipify, no torch cpp_extension).

Two shared objects are produced next to this file:

* ``_twtml_host*.so`` — host C++17 runtime (synthetic source, Unicode
  lowering, CPU featurizer), built with g++.
* ``_twtml_hip*.so`` — the MI355X engine: hand-written CDNA4 HIP kernels for
  gfx950 plus the C++ micro-batch engine and the RCCL communicator, built with
  ``hipcc --offload-arch=gfx950``.  It links the HIP runtime and RCCL that the
  installed PyTorch ships (``torch/lib``), so a process that imports torch
  and this extension holds ONE HIP runtime (same SONAMEs).

Builds are incremental (mtime based) and parallel per translation unit.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys
import sysconfig
from typing import List, Optional, Sequence

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
BUILD_DIR = os.path.join(ROOT, "build", "native")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = os.environ.get("TWTML_OFFLOAD_ARCH", "gfx950")

HOST_SO = os.path.join(PKG_DIR, "_twtml_host" + EXT)
HIP_SO = os.path.join(PKG_DIR, "_twtml_hip" + EXT)


def _pybind_includes() -> List[str]:
    import pybind11
    return [pybind11.get_include(), sysconfig.get_paths()["include"]]


def _torch_lib_dir() -> Optional[str]:
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec is None or not spec.submodule_search_locations:
            return None
        d = os.path.join(list(spec.submodule_search_locations)[0], "lib")
        return d if os.path.isdir(d) else None
    except Exception:  # pragma: no cover
        return None


def _newer(target: str, deps: Sequence[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _headers(*dirs: str) -> List[str]:
    out: List[str] = []
    for d in dirs:
        out += glob.glob(os.path.join(d, "*.h"))
    return out


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print("+", " ".join(cmd), flush=True)
    res = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"native build failed ({res.returncode}):\n{' '.join(cmd)}\n{res.stdout}")
    if verbose and res.stdout.strip():
        print(res.stdout, flush=True)


def build_host(force: bool = False, verbose: bool = False) -> str:
    srcs = sorted(glob.glob(os.path.join(CSRC, "host", "*.cpp")))
    deps = srcs + _headers(os.path.join(CSRC, "host"), os.path.join(CSRC, "common"))
    if not force and not _newer(HOST_SO, deps):
        return HOST_SO
    cxx = os.environ.get("CXX", "g++")
    os.makedirs(BUILD_DIR, exist_ok=True)
    inc = [f"-I{p}" for p in _pybind_includes()]
    objs = []

    def compile_one(src: str) -> str:
        obj = os.path.join(BUILD_DIR, "host_" + os.path.basename(src) + ".o")
        if force or _newer(obj, [src] + deps[len(srcs):]):
            _run([cxx, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", "-Wall",
                  "-Wno-unused-function", *inc, "-c", src, "-o", obj], verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, srcs))
    tmp = HOST_SO + ".tmp"
    _run([cxx, "-shared", "-o", tmp, *objs, "-lpthread"], verbose)
    os.replace(tmp, HOST_SO)
    return HOST_SO


def hipcc() -> str:
    p = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    if not os.path.exists(p):
        raise RuntimeError("hipcc not found; set ROCM_PATH")
    return p


HIP_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
             "-ffp-contract=fast", "-Wno-unused-result"]
# Per-source extras.  kmeans.hip: MFMA accumulators in VGPRs (the k-means
# assignment reads every accumulator on the VALU after each tile; AGPR
# accumulators cost a v_accvgpr_read per value -- 16 of ~128 VALU per tile).
HIP_FILE_FLAGS = {"kmeans.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}


def build_hip(force: bool = False, verbose: bool = False) -> str:
    """Compile csrc/hip/*.hip (device) + *.cpp (host engine) into _twtml_hip."""
    hip_dir = os.path.join(CSRC, "hip")
    kern = sorted(glob.glob(os.path.join(hip_dir, "*.hip")))
    host = sorted(glob.glob(os.path.join(hip_dir, "*.cpp")))
    hdrs = _headers(hip_dir, os.path.join(CSRC, "common"))
    deps = kern + host + hdrs
    if not kern:
        raise RuntimeError("no HIP sources")
    if not force and not _newer(HIP_SO, deps):
        return HIP_SO
    os.makedirs(BUILD_DIR, exist_ok=True)
    cc = hipcc()
    inc = [f"-I{p}" for p in _pybind_includes()] + [f"-I{ROCM}/include", f"-I{CSRC}"]

    def compile_one(src: str) -> str:
        obj = os.path.join(BUILD_DIR, "hip_" + os.path.basename(src) + ".o")
        if force or _newer(obj, [src] + hdrs):
            extra = ["-x", "hip"] if src.endswith(".hip") else ["-x", "c++", "-D__HIP_PLATFORM_AMD__"]
            if src.endswith(".cpp"):
                cmd = [cc, "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden", *inc, *extra,
                       "-c", src, "-o", obj]
            else:
                cmd = [cc, *HIP_FLAGS, *HIP_FILE_FLAGS.get(os.path.basename(src), []), "-fvisibility=hidden",
                       *inc, *extra, "-c", src, "-o", obj]
            _run(cmd, verbose)
        return obj

    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        objs = list(ex.map(compile_one, kern + host))
    tl = _torch_lib_dir()
    link = [cc, "-shared", f"--offload-arch={ARCH}", "-o", HIP_SO + ".tmp", *objs]
    if tl and os.path.exists(os.path.join(tl, "libamdhip64.so")):
        # bind to torch's runtime + RCCL so one process never holds two copies
        link += [os.path.join(tl, "libamdhip64.so"), os.path.join(tl, "librccl.so"),
                 f"-Wl,-rpath,{tl}"]
    else:
        link += [f"-L{ROCM}/lib", "-lamdhip64", "-lrccl", f"-Wl,-rpath,{ROCM}/lib"]
    link += [f"-L{ROCM}/lib", "-lrocprofiler-sdk-roctx", f"-Wl,-rpath,{ROCM}/lib", "-lpthread"]
    _run(link, verbose)
    os.replace(HIP_SO + ".tmp", HIP_SO)
    return HIP_SO


def build_all(force: bool = False, verbose: bool = False, hip: bool = True) -> None:
    build_host(force, verbose)
    if hip:
        build_hip(force, verbose)


def main(argv=None) -> int:
    """``twtml-build [--force] [-v] [--host-only]``: compile the in-tree extensions."""
    argv = sys.argv[1:] if argv is None else argv
    build_all(force="--force" in argv, verbose="-v" in argv or "--verbose" in argv,
              hip="--host-only" not in argv)
    return 0


if __name__ == "__main__":
    sys.exit(main())
