"""Build an alternative copy of the extension for same-box A/B runs (load it with
CASSMANTLE_EXT_SO=<out>): the in-tree objects of ``build/hip`` are reused, only the named
translation units are recompiled with extra flags and/or from another source file.

    python tools/build_variant.py OUT.so [--file gemm_areg.hip] [--flags "-fno-slp-vectorize"]
                                          [--src path/to/alternative/gemm_areg.hip]
"""
import argparse
import glob
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd import build as B  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--file", action="append", default=[], help="translation unit to rebuild (basename)")
    ap.add_argument("--flags", default="", help="extra hipcc flags for the rebuilt units")
    ap.add_argument("--src", action="append", default=[], help="alternative source per --file (same order)")
    a = ap.parse_args()
    B.build()                                  # the in-tree objects are current
    hipcc = B._hipcc()
    objs = []
    vdir = os.path.join(B.BUILD, "variant")
    os.makedirs(vdir, exist_ok=True)
    srcs = dict(zip(a.file, a.src))
    cmds = []
    for src in sorted(glob.glob(os.path.join(B.CSRC, "*.hip"))):
        name = os.path.basename(src)
        obj = os.path.join(B.BUILD, name + ".o")
        if name in a.file:
            alt = srcs.get(name, src)
            obj = os.path.join(vdir, name + ".o")
            cmds.append([hipcc, f"--offload-arch={B.ARCH}", "-munsafe-fp-atomics", "-O3", "-fPIC", "-std=c++17",
                         f"-I{B.CSRC}", "-Wno-unused-result", "-Wno-unused-variable", "-mllvm",
                         "-pragma-unroll-threshold=100000", *a.flags.split(), "-c", alt, "-o", obj])
        objs.append(obj)
    import concurrent.futures as cf
    with cf.ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:   # the rebuilt units in parallel
        for r in ex.map(lambda c: subprocess.run(c, check=True), cmds):
            pass
    objs.append(os.path.join(B.BUILD, "bindings.o"))
    _, lib, _ = B._torch_paths()
    subprocess.run([hipcc, "-shared", "-fPIC", f"--offload-arch={B.ARCH}", *objs, "-o", a.out, f"-L{lib}", "-lc10",
                    "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-ltorch_python", f"-Wl,-rpath,{lib}"],
                   check=True)
    print(a.out)


if __name__ == "__main__":
    main()
