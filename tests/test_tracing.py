"""Per-stage tracing: histogram semantics, Prometheus rendering, host spans, the
pipeline's encode/denoise/decode spans and the scorer's spans reaching /metrics."""
import asyncio

import numpy as np
import pytest
import torch

from cassmantle_amd.utils.tracing import Histogram, Tracer, TRACER


def test_histogram_buckets_are_cumulative():
    h = Histogram("x", buckets=(1, 10, 100))
    for v in (0.5, 1.0, 5, 50, 500):
        h.observe(v)
    lines = h.render("m")
    assert 'm_bucket{stage="x",le="1"} 2' in lines          # le is inclusive
    assert 'm_bucket{stage="x",le="10"} 3' in lines
    assert 'm_bucket{stage="x",le="100"} 4' in lines
    assert 'm_bucket{stage="x",le="+Inf"} 5' in lines
    assert 'm_count{stage="x"} 5' in lines
    assert h.percentile(50) == 5 and h.max == 500


def test_host_span_and_snapshot():
    t = Tracer()
    for _ in range(3):
        with t.span("work"):
            sum(range(1000))
    snap = t.snapshot()
    assert snap["work"]["count"] == 3 and snap["work"]["sum_ms"] >= 0
    text = t.render_prometheus()
    assert "# TYPE cassmantle_stage_ms histogram" in text
    assert 'cassmantle_stage_ms_count{stage="work"} 3' in text


def test_disabled_tracer_records_nothing():
    t = Tracer(enabled=False)
    with t.span("a"):
        pass
    t.observe("b", 1.0)
    assert t.snapshot() == {}


def test_span_records_even_when_region_raises():
    t = Tracer()
    with pytest.raises(ValueError):
        with t.span("boom"):
            raise ValueError
    assert t.snapshot()["boom"]["count"] == 1


def test_tiny_pipeline_records_stages_on_cpu():
    from cassmantle_amd import ops
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    ops.set_mode("torch")
    TRACER.reset()
    sd = StableDiffusion(SPECS["tiny"], device="cpu", dtype=torch.float32)
    sd.generate_tensor(["a lantern"], "blurry", [0], steps=2)
    snap = TRACER.snapshot()
    for st in ("encode", "denoise", "decode"):
        assert snap[st]["count"] == 1, snap


def test_scorer_spans_reach_metrics_endpoint():
    from test_api import make_client
    TRACER.reset()
    client, svc = make_client()
    with client:
        client.get("/init")
        secret = svc.room("").fetch_current_prompt()
        m0 = secret["masks"][0]
        client.post("/compute_score", json={"inputs": {str(m0): "lantern"}})
        client.get("/fetch/contents")
        text = client.get("/metrics").text
        assert 'cassmantle_stage_ms_count{stage="score_request"}' in text
        assert 'cassmantle_stage_ms_count{stage="score_batch"}' in text
        assert "stages" in client.get("/healthz").json()


@pytest.mark.gpu
def test_gpu_span_uses_device_events_without_sync():
    t = Tracer()
    s = torch.cuda.Stream()
    a = torch.randn(2048, 2048, device="cuda", dtype=torch.bfloat16)
    with torch.cuda.stream(s):
        with t.span("mm", s):
            for _ in range(4):
                a = a @ a.T * 1e-3
    t.flush()
    snap = t.snapshot()
    assert snap["mm"]["count"] == 1 and snap["mm"]["sum_ms"] > 0
