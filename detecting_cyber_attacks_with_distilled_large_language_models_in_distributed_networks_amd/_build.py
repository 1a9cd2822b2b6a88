"""In-tree native build: gfx950 HIP kernel library + torch binding, and the C++ text front-end.

Outputs (git-ignored, but shipped to the GPU box with the repo snapshot):
  ops/_hip_kernels<EXT_SUFFIX>      csrc/kernels/*.hip (hipcc --offload-arch=gfx950) + csrc/comm/*.cpp
                                    (native RCCL communicator) + csrc/binding.cpp
  data/_text_native_impl<EXT_SUFFIX> csrc/text/text_native.cpp (g++, pybind11)

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
BUILD = os.path.join(REPO, "build", "native")
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_OUT = os.path.join(PKG_DIR, "ops", "_hip_kernels" + EXT)
TEXT_OUT = os.path.join(PKG_DIR, "data", "_text_native_impl" + EXT)


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
                               "-munsafe-fp-atomics", "-I" + kdir, "-c", s, "-o", o], o))
    for s in sorted(glob.glob(os.path.join(CSRC, "comm", "*.cpp"))):
        o = os.path.join(BUILD, "comm_" + os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s]):
            jobs_list.append(([HIPCC, "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-c", s, "-o", o], o))
    inc, defs, libdir = _torch_flags()
    bo = os.path.join(BUILD, "binding.o")
    objs.append(bo)
    if force or _newer(bo, [binding]):
        jobs_list.append(([HIPCC, "-O2", "-std=c++17", "-fPIC", "-w"] + defs + ["-I" + i for i in inc]
                          + ["-c", binding, "-o", bo], bo))
    if jobs_list:
        n = jobs or min(8, len(jobs_list))
        with ThreadPoolExecutor(n) as ex:
            list(ex.map(lambda j: _run(j[0], verbose), jobs_list))
    if force or jobs_list or _newer(HIP_OUT, objs):
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
