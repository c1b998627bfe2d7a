"""ISA guard of the in-kernel LayerNorm / GroupNorm race fix (CPU, hipcc only).

The round-2 race (whole 16-row groups of the A-in-registers GEMM with wrong LayerNorm
statistics, only while another kernel shared the CU) needed packed fp32 (``v_pk_*_f32``,
produced by SLP vectorisation) in the statistics prologue, read back at the compiler's minimum
hazard distance (``profiles/r3_lnk_race_rootcause.txt``; note in ``ops/csrc/gemm_areg.hip``
above ``sum_row_groups``).  The fix lives in the source: the prologue is scalar fp32 and is
finished before the first LDS-DMA.  Nothing in the compiler keeps it that way, so this test
disassembles every LNK / GNK instantiation of ``gemm_areg_kernel`` and fails if a packed-fp32
instruction appears before the kernel's first ``buffer_load ... lds``.

Checked both ways: the round-2 source (commit 02d221a, ``gemm_areg.hip`` with its headers)
built with the default flags has packed fp32 ahead of the first DMA in its LNK kernels, and
fails; the current source passes."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cassmantle_amd", "ops", "csrc")
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)

NAME = re.compile(r"^(_Z\S*?gemm_areg_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELb([01])ELb([01])(?:ELb([01]))?E\S*):", re.M)
PK_F32 = re.compile(r"^\s*v_pk_(?:add|mul|fma|mov)_[fb]32\b")
DMA = re.compile(r"^\s*buffer_load_\w+.*\blds\b")


def compile_asm(src: str, csrc: str, out: str) -> str:
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-I", csrc, "-mllvm",
                        "-pragma-unroll-threshold=100000", "--cuda-device-only", "-S", src, "-o", out],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    return open(out).read()


def packed_before_first_dma(asm: str):
    """-> {kernel: [packed-fp32 instructions ahead of its first LDS-DMA]} for the LNK / GNK
    instantiations (template flags 6 and 7), and the number of such kernels seen."""
    bad, seen = {}, 0
    for m in NAME.finditer(asm):
        lnk, gnk = m.group(7) == "1", m.group(8) == "1"      # (GNK: absent before round 3)
        if not (lnk or gnk):
            continue
        seen += 1
        body = asm[m.end():asm.find(".Lfunc_end", m.end())]
        pre = []
        for line in body.splitlines():
            if DMA.match(line):
                break
            if PK_F32.match(line):
                pre.append(line.strip())
        if pre:
            bad[m.group(1)] = pre
    return bad, seen


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
def test_norm_prologue_has_no_packed_fp32_before_first_dma():
    out = os.path.join(ROOT, "build", "isacheck", "gemm_areg.s")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    asm = compile_asm(os.path.join(CSRC, "gemm_areg.hip"), CSRC, out)
    bad, seen = packed_before_first_dma(asm)
    assert seen >= 4, "no LNK / GNK instantiations found: the name pattern is stale"
    assert bad == {}, {k: v[:4] for k, v in bad.items()}
