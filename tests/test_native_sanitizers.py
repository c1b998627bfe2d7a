"""Host-side sanitizer runs of the native GEMM planner / tuning table.

tests/native/planner_sanitize.cpp is linked against ops/csrc/gemm.hip + gemm_areg.hip (tile
launchers stubbed) and built twice with hipcc, sanitizers on the HOST side only
(``-Xarch_host -fsanitize=...``; GPU sanitizers are not available on this pool): ASan + UBSan,
and TSan.  The driver plans GEMMs from 4 threads while the tuning table is loaded and cleared --
what serving does with the generation and scorer threads -- and checks determinism.  Runs on
the CPU (nothing is launched); the TSan build is what flagged the planner's process-global
"last plan" state, now thread-local."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "cassmantle_amd", "ops", "csrc")
DRIVER = os.path.join(ROOT, "tests", "native", "planner_sanitize.cpp")
OUT = os.path.join(ROOT, "build", "native")
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)
SRCS = [os.path.join(CSRC, "gemm.hip"), os.path.join(CSRC, "gemm_areg.hip"), DRIVER]


def _build(name, flags):
    os.makedirs(OUT, exist_ok=True)
    exe = os.path.join(OUT, name)
    deps = SRCS + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")]
    if os.path.exists(exe) and os.path.getmtime(exe) > max(os.path.getmtime(d) for d in deps):
        return exe
    cmd = [HIPCC, "--offload-arch=gfx950", "-O1", "-g", "-std=c++17", "-I", CSRC, *flags, *SRCS, "-o", exe,
           "-mllvm", "-pragma-unroll-threshold=100000"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


@pytest.mark.skipif(HIPCC is None, reason="hipcc not available")
@pytest.mark.parametrize("name,flags", [
    ("planner_asan", ["-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                      "-Xarch_host", "-fno-omit-frame-pointer", "-Xarch_host", "-fno-sanitize-recover=undefined"]),
    ("planner_tsan", ["-Xarch_host", "-fsanitize=thread"]),
])
def test_planner_under_host_sanitizers(name, flags):
    exe = _build(name, flags)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=0:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "mismatches 0" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
