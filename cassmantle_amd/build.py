"""Ahead-of-time build of the in-tree HIP extension (``cassmantle_amd/_C*.so``) for gfx950.

Kernel translation units (``ops/csrc/*.hip``) are compiled by ``hipcc --offload-arch=gfx950``
without any torch headers (seconds each, rebuilt only when they or a header change); the single
``bindings.cpp`` is the only unit that includes libtorch.  Objects are linked into one shared
object placed inside the package, so it travels with the repository snapshot to the GPU box and
shows up as in-tree native code when loaded.  No hipify step, no JIT cache.

    python -m cassmantle_amd.build [--force] [--jobs N] [--verbose]
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
from typing import List

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "ops", "csrc")
BUILD = os.path.join(os.path.dirname(PKG), "build", "hip")
ARCH = os.environ.get("CASSMANTLE_ARCH", "gfx950")


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found")


def _torch_paths():
    import torch
    from torch.utils import cpp_extension as ce
    inc = ce.include_paths(device_type="cuda") if "device_type" in ce.include_paths.__code__.co_varnames \
        else ce.include_paths(True)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return inc, lib, abi


def _newer(src: str, dst: str, deps: List[str]) -> bool:
    if not os.path.exists(dst):
        return True
    t = os.path.getmtime(dst)
    return any(os.path.getmtime(s) > t for s in [src] + deps)


def target_path() -> str:
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(PKG, "_C" + suffix)


def build(force: bool = False, jobs: int = 0, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    hipcc = _hipcc()
    headers = glob.glob(os.path.join(CSRC, "*.h"))
    hip_srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    binding = os.path.join(CSRC, "bindings.cpp")
    inc, lib, abi = _torch_paths()
    py_inc = sysconfig.get_paths()["include"]
    # -pragma-unroll-threshold: the GEMM epilogues fully unroll over up to 32 accumulator
    # fragments; past the default limit the unroller gives up and the accumulators go to scratch
    common = ["-O3", "-fPIC", "-std=c++17", f"-I{CSRC}", "-Wno-unused-result", "-Wno-unused-variable",
              "-mllvm", "-pragma-unroll-threshold=100000"]
    # per-file extra flags (none: the in-kernel LayerNorm's permlane hazard is padded in the
    # source, gemm_areg.hip sum_row_groups, instead of by building that file without SLP)
    file_flags: dict = {}
    cmds = []
    objs = []
    for src in hip_srcs:
        obj = os.path.join(BUILD, os.path.basename(src) + ".o")
        objs.append(obj)
        if force or _newer(src, obj, headers):
            cmds.append([hipcc, f"--offload-arch={ARCH}", "-munsafe-fp-atomics", *common,
                         *file_flags.get(os.path.basename(src), []), "-c", src, "-o", obj])
    bobj = os.path.join(BUILD, "bindings.o")
    objs.append(bobj)
    if force or _newer(binding, bobj, headers):
        tflags = [f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DTORCH_API_INCLUDE_EXTENSION_H", "-DTORCH_EXTENSION_NAME=_C",
                  "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2"]
        incs = [f"-I{p}" for p in inc] + [f"-I{py_inc}"]
        cmds.append([hipcc, f"--offload-arch={ARCH}", *common, "-O2", *tflags, *incs, "-c", binding, "-o", bobj])
    jobs = jobs or min(8, os.cpu_count() or 4)

    def run(cmd):
        if verbose:
            print(" ".join(cmd), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        return cmd[-1]

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        for out in ex.map(run, cmds):
            if verbose:
                print("built", out, flush=True)
    target = target_path()
    if force or cmds or not os.path.exists(target):
        link = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", target + ".tmp",
                f"-L{lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python",
                f"-Wl,-rpath,{lib}"]
        run(link)
        os.replace(target + ".tmp", target)
    return target


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--jobs", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    a = ap.parse_args(argv)
    print(build(a.force, a.jobs, a.verbose))
    return 0


if __name__ == "__main__":
    sys.exit(main())
