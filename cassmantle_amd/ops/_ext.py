"""Loader for the in-tree HIP extension ``cassmantle_amd/_C*.so``.

The extension is built ahead of time (``python -m cassmantle_amd.build``; also run by
``__graft_entry__.build()``) so the shared object ships inside the repository snapshot to the
GPU box.  Import is lazy: importing the package on a CPU-only host never touches HIP.
"""
from __future__ import annotations

import glob
import importlib.util
import os
import sys
from typing import Optional

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ext = None
_err: Optional[str] = None
_tried = False


def so_path() -> Optional[str]:
    # CASSMANTLE_EXT_SO: load another build of the extension (same-box A/B of compile options)
    alt = os.environ.get("CASSMANTLE_EXT_SO") or None
    if alt:
        return alt
    cands = sorted(glob.glob(os.path.join(_PKG, "_C*.so")))
    return cands[0] if cands else None


def _load():
    global _ext, _err, _tried
    _tried = True
    path = so_path()
    if path is None:
        _err = "extension _C*.so not built"
        return
    try:
        import torch  # noqa: F401  - libtorch/libamdhip64 must be loaded first
        spec = importlib.util.spec_from_file_location("cassmantle_amd._C", path)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        sys.modules["cassmantle_amd._C"] = mod
        _ext = mod
    except Exception as e:  # noqa: BLE001
        _err = f"failed to load {path}: {e}"


def ext():
    if not _tried:
        _load()
    if _ext is None:
        raise RuntimeError(_err or "extension unavailable")
    return _ext


def ext_available() -> bool:
    if not _tried:
        _load()
    return _ext is not None


def ext_error() -> Optional[str]:
    return _err
