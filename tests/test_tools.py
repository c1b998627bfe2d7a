"""CPU tests of the tuning tools' host logic (tools/autotune_gemm.py --cold weight rotation) and of
the scorer stream-priority wiring (config.ModelConfig.scorer_stream_priority)."""
import importlib
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _autotune():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    try:
        return importlib.import_module("autotune_gemm")
    finally:
        sys.path.pop(0)


def _recorded(fn, *args, **kw):
    call = lambda: fn(*args, **kw)   # noqa: E731 - the shape ops._launch records
    call.fn, call.args, call.kw = fn, args, kw
    return call


def test_cold_rotation_swaps_only_the_weight():
    at = _autotune()
    seen = []
    x = torch.zeros(4, 8, dtype=torch.bfloat16)
    w = torch.zeros(16, 8, dtype=torch.bfloat16)
    b = torch.zeros(16, dtype=torch.bfloat16)
    call = _recorded(lambda x_, w_, b_, act=0: seen.append((x_.data_ptr(), w_.data_ptr(), b_.data_ptr(), act)),
                     x, w, b, act=3)
    run = at.weight_rotation("m4 n16 k8 w16 b1 c0:0:0:0:1:1:0:0", call, 1)
    for _ in range(6):
        run()
    assert len(run.copies) >= 2
    assert all(s[0] == x.data_ptr() and s[2] == b.data_ptr() and s[3] == 3 for s in seen)   # x / bias / kwargs kept
    assert len({s[1] for s in seen}) == min(6, len(run.copies)) and w.data_ptr() not in {s[1] for s in seen}


def test_cold_rotation_declines_an_ambiguous_or_missing_weight():
    at = _autotune()
    x = torch.zeros(16, 8, dtype=torch.bfloat16)
    w = torch.zeros(16, 8, dtype=torch.bfloat16)
    w2 = torch.zeros(16, 8, dtype=torch.bfloat16)
    assert at.weight_rotation("m16 n16 k8 w16", _recorded(lambda *a: None, x, w, w2), 1) is None   # two candidates
    assert at.weight_rotation("m16 n16 k8 w32", _recorded(lambda *a: None, x, w), 1) is None       # no Nw x K tensor
    assert at.weight_rotation("m16 n16 k8 w16", lambda: None, 1) is None                          # not a recorded call


def test_scorer_stream_priority_config():
    from cassmantle_amd.config import Config
    cfg = Config()
    assert cfg.model.scorer_stream_priority is None      # auto: -1 in-process, 0 in the supervised front-end
    src = open(os.path.join(ROOT, "cassmantle_amd", "serve.py")).read()
    assert "cfg.model.scorer_stream_priority = 0" in src
