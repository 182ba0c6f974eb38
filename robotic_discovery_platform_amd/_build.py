"""In-tree native build: HIP kernels (hipcc --offload-arch=gfx950) + C++ runtime + torch bindings.

No hipify, no torch.utils.cpp_extension JIT: every ``csrc/*.hip`` is compiled by hipcc for gfx950
only, ``csrc/*.cpp`` host sources by g++, and everything is linked into
``robotic_discovery_platform_amd/_C.so`` (ships to the GPU box with the repo snapshot).
Incremental on mtimes (headers are a dependency of every source).

Usage: ``python -m robotic_discovery_platform_amd._build [--force] [-j N]``
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig
import time

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "obj")
OUT = os.path.join(PKG_DIR, "_C.so")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _torch_paths():
    import torch
    tdir = os.path.dirname(torch.__file__)
    inc = [os.path.join(tdir, "include"), os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    return inc, os.path.join(tdir, "lib"), int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _newest(paths):
    return max((os.path.getmtime(p) for p in paths if os.path.exists(p)), default=0.0)


def _run(cmd):
    t0 = time.time()
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}")
    return time.time() - t0, r.stdout


def host_sources():
    return sorted(p for p in glob.glob(os.path.join(CSRC, "*.cpp")))


def hip_sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")))


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hdr_time = _newest(headers)
    tinc, tlib, abi = _torch_paths()
    pyinc = sysconfig.get_paths()["include"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    tasks = []
    objs = []
    for src in hip_sources():
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_time):
            tasks.append([os.path.join(ROCM, "bin", "hipcc"), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC",
                          "-ffp-contract=fast", "-munsafe-fp-atomics", "-I", CSRC, "-c", src, "-o", obj])
    for src in host_sources():
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or not os.path.exists(obj) or os.path.getmtime(obj) < max(os.path.getmtime(src), hdr_time):
            is_binding = os.path.basename(src) in ("bindings.cpp", "serve_runtime.cpp")  # pybind11 sources
            cmd = ["g++", "-O3", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
                   f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", CSRC, "-I", os.path.join(ROCM, "include")]
            if is_binding:
                cmd += ["-DTORCH_EXTENSION_NAME=_C"] + sum((["-I", p] for p in tinc), []) + ["-I", pyinc]
            cmd += ["-c", src, "-o", obj]
            tasks.append(cmd)
    if tasks:
        with cf.ThreadPoolExecutor(jobs) as ex:
            for cmd, (dt, _) in zip(tasks, ex.map(_run, tasks)):
                if verbose:
                    print(f"[rdp build] {os.path.basename(cmd[-3])}  {dt:.1f}s", flush=True)
    if force or tasks or not os.path.exists(OUT) or os.path.getmtime(OUT) < _newest(objs):
        link = ["g++", "-shared", "-o", OUT] + objs + [
            f"-L{tlib}", f"-L{os.path.join(ROCM, 'lib')}", f"-Wl,-rpath,{tlib}", f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}",
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", "-lamdhip64", "-lz"]
        _run(link)
        if verbose:
            print(f"[rdp build] linked {OUT}", flush=True)
    return OUT


if __name__ == "__main__":
    force = "--force" in sys.argv
    j = None
    if "-j" in sys.argv:
        j = int(sys.argv[sys.argv.index("-j") + 1])
    build(force=force, jobs=j)
