"""Register-pressure guard (CPU, hipcc only): the default GEMM / attention instantiations must not
spill to scratch.  An epilogue change once pushed the 256x256 ping-pong tiles to 256 VGPRs + 360 B
of scratch per lane and the VAE convs ran 7-10x slower on the GPU while every numerics test
passed (round 3, LayerNorm row statistics); this catches that class on the CPU."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cassmantle_amd", "ops", "csrc")
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)

# kernels that may spill (opt-in variants / knobs, documented where they are instantiated)
ALLOWED = ("gemm_areg_kernelILi20ELi2ELi2ELi2ELb0",)    # K = 640 ring-2 tiles (28-36 B, measured, default)


def _scratch(tu):
    out = os.path.join(ROOT, "build", "regcheck", tu + ".s")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", CSRC, "-mllvm",
                        "-pragma-unroll-threshold=100000", "--cuda-device-only", "-S",
                        os.path.join(CSRC, tu + ".hip"), "-o", out], capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    s = open(out).read()
    bad = []
    for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)\.vgpr_count:\s+(\d+)", s, re.S):
        pr = re.search(r"private_segment_fixed_size:\s+(\d+)", m.group(2))
        if pr and int(pr.group(1)) > 0 and not any(a in m.group(1) for a in ALLOWED):
            bad.append((m.group(1), int(m.group(3)), int(pr.group(1))))
    return bad


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
@pytest.mark.parametrize("tu", ["gemm_pp_c2", "gemm_pp_c0", "gemm_c0_buf", "gemm_areg", "attention", "norm"])
def test_default_kernels_do_not_spill(tu):
    assert _scratch(tu) == []
