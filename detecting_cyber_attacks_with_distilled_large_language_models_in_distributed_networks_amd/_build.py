"""In-tree native build: gfx950 HIP kernel library + torch binding, and the C++ text front-end.

Outputs (git-ignored, but shipped to the GPU box with the repo snapshot), both in
``<repo>/_so/`` -- a short path on purpose: the full package path made a mapped
library's /proc/<pid>/maps line ~260 characters long, which the GPU driver's
loaded-library audit dropped (GPUTEST_r01: native_lines_dropped=6):
  _so/_hip_kernels.so        csrc/kernels/*.hip (hipcc --offload-arch=gfx950) + csrc/comm/*.cpp
                             (native RCCL communicator) + csrc/binding.cpp
  _so/_text_native_impl.so   csrc/text/text_native.cpp (g++, pybind11)
They are imported as ``<pkg>.ops._hip_kernels`` / ``<pkg>.data._text_native_impl``
by ``load_extension`` (an ExtensionFileLoader on the explicit path).

Kernel objects compile in parallel and are rebuilt only when a source (or the
shared header) is newer than the object.  Usage: ``python -m <pkg>._build``.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(PKG_DIR)
CSRC = os.path.join(REPO, "csrc")
# experiment builds keep their objects apart (FD_BUILD_TAG=stamps -> build/native_stamps)
BUILD = os.path.join(REPO, "build", "native" + ("_" + os.environ["FD_BUILD_TAG"] if os.environ.get("FD_BUILD_TAG") else ""))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# experiment builds only (e.g. "-DFD_GEMM_SCHED=0"); use with force=True / a clean build dir
EXTRA = os.environ.get("FD_HIP_EXTRA_FLAGS", "").split()

SO_DIR = os.path.join(REPO, "_so")
# FD_SO_OUT: write (and load) the kernel library elsewhere, e.g. ab/stamps.so for a diagnostic build
HIP_OUT = os.environ.get("FD_SO_OUT") or os.path.join(SO_DIR, "_hip_kernels.so")
TEXT_OUT = os.path.join(SO_DIR, "_text_native_impl.so")


def load_extension(qualname: str, path: str):
    """Import the extension module ``qualname`` (PyInit_<last component>) from ``path``."""
    import importlib.machinery
    import importlib.util
    if qualname in sys.modules:
        return sys.modules[qualname]
    if not os.path.exists(path):
        raise ImportError(f"native extension not built: {path}")
    loader = importlib.machinery.ExtensionFileLoader(qualname, path)
    spec = importlib.util.spec_from_file_location(qualname, path, loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    sys.modules[qualname] = mod
    return mod


def load_hip():
    return load_extension(__package__ + ".ops._hip_kernels", HIP_OUT)


def load_text():
    return load_extension(__package__ + ".data._text_native_impl", TEXT_OUT)


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose=False):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build_text(verbose=False, force=False) -> str:
    src = os.path.join(CSRC, "text", "text_native.cpp")
    if not force and not _newer(TEXT_OUT, [src, os.path.join(CSRC, "text", "text_core.h")]):
        return TEXT_OUT
    import pybind11
    os.makedirs(SO_DIR, exist_ok=True)
    cmd = ["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread",
           "-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"],
           src, "-o", TEXT_OUT + ".tmp"]
    _run(cmd, verbose)
    os.replace(TEXT_OUT + ".tmp", TEXT_OUT)
    return TEXT_OUT


def _torch_flags():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
           sysconfig.get_paths()["include"]]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = ["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DTORCH_EXTENSION_NAME=_hip_kernels",
            "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}"]
    libdir = os.path.join(tdir, "lib")
    return inc, defs, libdir


def build_hip(verbose=False, force=False, jobs=None) -> str:
    kdir = os.path.join(CSRC, "kernels")
    sources = sorted(glob.glob(os.path.join(kdir, "*.hip")))
    headers = sorted(glob.glob(os.path.join(kdir, "*.h")))
    binding = os.path.join(CSRC, "binding.cpp")
    os.makedirs(BUILD, exist_ok=True)
    objs = []
    jobs_list = []
    for s in sources:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + headers):
            jobs_list.append(([HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                               "-munsafe-fp-atomics", "-I" + kdir] + EXTRA + ["-c", s, "-o", o], o))
    for s in sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp"))):
        o = os.path.join(BUILD, "comm_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s]):
            jobs_list.append(([HIPCC, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-c", s, "-o", o], o))
    inc, defs, libdir = _torch_flags()
    bo = os.path.join(BUILD, "binding.o")
    objs.append(bo)
    if force or _newer(bo, [binding] + headers):
        jobs_list.append(([HIPCC, "-O2", "-std=c++17", "-fPIC", "-w"] + defs + ["-I" + i for i in inc]
                          + ["-c", binding, "-o", bo], bo))
    if jobs_list:
        n = jobs or min(8, len(jobs_list))
        with ThreadPoolExecutor(n) as ex:
            list(ex.map(lambda j: _run(j[0], verbose), jobs_list))
    if force or jobs_list or _newer(HIP_OUT, objs):
        os.makedirs(os.path.dirname(HIP_OUT), exist_ok=True)
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + [
            "-L" + libdir, "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
            "-ldl",  # RCCL is bound at run time from torch's copy (csrc/comm/rccl_comm.cpp)
            "-Wl,-rpath," + libdir, "-o", HIP_OUT + ".tmp"]
        _run(cmd, verbose)
        os.replace(HIP_OUT + ".tmp", HIP_OUT)
    return HIP_OUT


def build_all(verbose=False, force=False):
    return build_text(verbose, force), build_hip(verbose, force)


if __name__ == "__main__":
    force = "--force" in sys.argv
    for p in build_all(verbose="-v" in sys.argv, force=force):
        print("built", p)
