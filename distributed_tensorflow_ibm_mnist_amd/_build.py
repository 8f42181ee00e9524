"""In-tree build of the native extensions (no hipify, no JIT cache).

* ``_kernels``  — HIP/CDNA4 kernels for gfx950 (``csrc/kernels/*.hip``, hipcc)
                 + torch binding (``csrc/binding.cpp``).
* ``_host``     — host-side C++ runtime (``csrc/host/*.cpp``): crc32c, TFRecord
                 reader/writer, tf.Example codec, tensor-bundle (SSTable) I/O,
                 IDX parsing.  Pure C++ (g++), usable on CPU-only machines.

The ``.so`` files land next to this file so they travel with the repo snapshot
to the GPU box.  Rebuilds are incremental (mtime based).

    python -m distributed_tensorflow_ibm_mnist_amd._build [--force] [--host-only]
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys
import sysconfig
from typing import List, Sequence

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("MNISTX_ARCH", "gfx950")
EXT_SUFFIX = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CXX = os.environ.get("CXX", "g++")


def _torch_paths():
    import torch.utils.cpp_extension as ce
    return ce.include_paths(), ce.library_paths()


def _newer(target: str, deps: Sequence[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")


def _headers(d: str) -> List[str]:
    out = []
    for base, _, files in os.walk(d):
        out += [os.path.join(base, f) for f in files if f.endswith((".h", ".hpp", ".cuh"))]
    return out


def kernels_so() -> str:
    return os.path.join(PKG, "_kernels" + EXT_SUFFIX)


def host_so() -> str:
    return os.path.join(PKG, "_host" + EXT_SUFFIX)


def build_host(force: bool = False, verbose: bool = True) -> str:
    """Host runtime: plain C++17 + pybind11 (no torch, no HIP)."""
    import pybind11
    srcs = sorted(os.path.join(CSRC, "host", f) for f in os.listdir(os.path.join(CSRC, "host")) if f.endswith(".cpp"))
    out = host_so()
    deps = srcs + _headers(os.path.join(CSRC, "host"))
    if not force and not _newer(out, deps):
        return out
    py_inc = sysconfig.get_paths()["include"]
    cmd = [CXX, "-std=c++17", "-O3", "-fPIC", "-shared", "-msse4.2", "-fvisibility=hidden",
           f"-I{py_inc}", f"-I{pybind11.get_include()}", f"-I{os.path.join(CSRC, 'host')}",
           *srcs, "-o", out, "-lpthread"]
    if verbose:
        print("[build] host runtime ->", os.path.relpath(out, ROOT), flush=True)
    _run(cmd)
    return out


def build_kernels(force: bool = False, verbose: bool = True, jobs: int = 8) -> str:
    inc, libs = _torch_paths()
    os.makedirs(BUILD, exist_ok=True)
    kdir = os.path.join(CSRC, "kernels")
    hip_srcs = sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))
    hdrs = _headers(kdir)
    objs = []
    jobs_list = []
    for s in hip_srcs:
        o = os.path.join(BUILD, os.path.basename(s) + ".o")
        objs.append(o)
        if force or _newer(o, [s] + hdrs):
            # MFMA accumulators in the VGPR form: the AGPR form made the register allocator
            # shuffle loop-carried accumulators with v_accvgpr moves (up to 12 per step)
            jobs_list.append([HIPCC, "-std=c++17", "-O3", f"--offload-arch={ARCH}", "-fno-gpu-rdc", "-fPIC",
                              "-mllvm", "-amdgpu-mfma-vgpr-form",
                              "-D__HIP_PLATFORM_AMD__=1", f"-I{CSRC}", "-c", s, "-o", o])
    bsrc = os.path.join(CSRC, "binding.cpp")
    bobj = os.path.join(BUILD, "binding.o")
    objs.append(bobj)
    if force or _newer(bobj, [bsrc] + hdrs):
        py_inc = sysconfig.get_paths()["include"]
        jobs_list.append([CXX, "-std=c++17", "-O2", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
                          "-DTORCH_EXTENSION_NAME=_kernels", "-DTORCH_API_INCLUDE_EXTENSION_H",
                          "-D_GLIBCXX_USE_CXX11_ABI=1", "-I/opt/rocm/include", f"-I{CSRC}", f"-I{py_inc}",
                          *[f"-I{p}" for p in inc], "-c", bsrc, "-o", bobj])
    if verbose and jobs_list:
        print(f"[build] compiling {len(jobs_list)} unit(s) for {ARCH} ...", flush=True)
    with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(jobs_list) or 1))) as ex:
        list(ex.map(_run, jobs_list))
    out = kernels_so()
    if force or jobs_list or _newer(out, objs):
        cmd = [HIPCC, "-shared", "-fPIC", "-fno-gpu-rdc", f"--offload-arch={ARCH}", *objs,
               *[f"-L{p}" for p in libs], *[f"-Wl,-rpath,{p}" for p in libs],
               "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lamdhip64", "-o", out]
        if verbose:
            print("[build] linking ->", os.path.relpath(out, ROOT), flush=True)
        _run(cmd)
    return out


def build_all(force: bool = False, verbose: bool = True) -> None:
    build_host(force, verbose)
    build_kernels(force, verbose)


if __name__ == "__main__":
    force = "--force" in sys.argv
    if "--host-only" in sys.argv:
        build_host(force)
    else:
        build_all(force)
