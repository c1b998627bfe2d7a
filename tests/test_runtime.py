"""Serving runtime on the CPU: config wiring (weights_path, dtype, batching knobs), the batching
image generator shared by rooms, the pipeline's generation lock, store thread safety and the
tracer's capture guard."""
import os
import threading
import time

import numpy as np
import pytest
import torch

from cassmantle_amd.config import Config
from cassmantle_amd.game.content import BatchingImageGenerator, ImageGenerationError, ImageGenerator, SolidImageGenerator
from cassmantle_amd.game.clock import FakeClock
from cassmantle_amd.game.store import StateStore


class _Recorder(ImageGenerator):
    resolution = 8

    def __init__(self, fail=False, delay=0.05):
        self.calls = []
        self.fail = fail
        self.delay = delay
        self.active = 0
        self.max_active = 0
        self._mu = threading.Lock()

    def generate(self, prompts, negative, seeds):
        with self._mu:
            self.active += 1
            self.max_active = max(self.max_active, self.active)
        try:
            self.calls.append(list(prompts))
            time.sleep(self.delay)
            if self.fail:
                raise ImageGenerationError("boom")
            return [np.full((8, 8, 3), s % 256, np.uint8) for s in seeds]
        finally:
            with self._mu:
                self.active -= 1


def _concurrent(gen, n, **kw):
    out, errs = [None] * n, [None] * n

    def run(i):
        try:
            out[i] = gen.generate([f"p{i}"], "neg", [i])
        except Exception as e:  # noqa: BLE001
            errs[i] = e
    ths = [threading.Thread(target=run, args=(i,)) for i in range(n)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=30)
    return out, errs


def test_batching_generator_batches_concurrent_rooms_and_routes_results():
    inner = _Recorder()
    gen = BatchingImageGenerator(inner, max_batch=4, window_s=0.05)
    out, errs = _concurrent(gen, 6)
    assert all(e is None for e in errs)
    for i, imgs in enumerate(out):                        # every room got ITS image
        assert len(imgs) == 1 and imgs[0][0, 0, 0] == i
    assert inner.max_active == 1                          # the device pipeline is never shared
    assert max(gen.batch_sizes) > 1 and sum(gen.batch_sizes) == 6
    assert all(b <= 4 for b in gen.batch_sizes)


def test_batching_generator_propagates_failure_to_every_room_of_the_batch():
    gen = BatchingImageGenerator(_Recorder(fail=True), max_batch=8, window_s=0.05)
    out, errs = _concurrent(gen, 3)
    assert all(isinstance(e, ImageGenerationError) for e in errs)


def test_pipeline_concurrent_generate_is_serialised_and_correct():
    """two rooms' threads driving ONE tiny pipeline at once get the same images as sequential
    calls (the per-pipeline lock keeps the shared step state from interleaving)"""
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    sd = StableDiffusion(SPECS["tiny"], device="cpu", use_graphs=False)
    ref = {i: sd.generate([f"prompt {i}"], "neg", [i], steps=2)[0] for i in range(2)}
    res = {}

    def run(i):
        res[i] = sd.generate([f"prompt {i}"], "neg", [i], steps=2)[0]
    ths = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=120)
    for i in range(2):
        assert np.array_equal(res[i], ref[i])
    assert sd.last_finite is not None and bool(sd.last_finite)


def test_nonfinite_latents_raise():
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    sd = StableDiffusion(SPECS["tiny"], device="cpu", use_graphs=False)
    with torch.no_grad():
        sd.unet.conv_out.bias.fill_(float("nan"))
    with pytest.raises(ImageGenerationError):
        sd.generate(["x"], "neg", [0], steps=2)


def test_weights_path_loads_a_diffusers_checkpoint(tmp_path):
    from safetensors.torch import save_file
    from cassmantle_amd.models.weights import export_diffusers
    from cassmantle_amd.pipeline import SPECS, DiffusionImageGenerator, StableDiffusion
    src = StableDiffusion(SPECS["tiny"], device="cpu", use_graphs=False, seed=7)
    for sub, model, kind in (("unet", src.unet, "unet"), ("vae", src.vae, "vae"),
                             ("text_encoder", src.text_encoders[0], "clip")):
        os.makedirs(tmp_path / sub)
        save_file(export_diffusers(model, kind), str(tmp_path / sub / "model.safetensors"))
    gen = DiffusionImageGenerator("tiny", device="cpu", use_graphs=False, seed=0, weights_path=str(tmp_path))
    assert gen.weights_loaded == {"unet": 0, "vae": 0, "text_encoder": 0}
    for a, b in ((src.unet, gen.sd.unet), (src.vae, gen.sd.vae), (src.text_encoders[0], gen.sd.text_encoders[0])):
        for (n, p), (_, q) in zip(a.state_dict().items(), b.state_dict().items()):
            assert torch.equal(p, q), n
    with pytest.raises(FileNotFoundError):
        DiffusionImageGenerator("tiny", device="cpu", use_graphs=False, weights_path=str(tmp_path / "nope"))


def test_config_dtype_and_factory_wiring():
    from cassmantle_amd.runtime.factory import build_service, model_dtype
    cfg = Config.from_args(["--dtype", "fp32", "--num_rooms", "3", "--gen_batch_max", "2"])
    assert model_dtype(cfg, "cpu") == torch.float32
    with pytest.raises(ValueError):
        model_dtype(cfg, "cuda")
    cfg.model.dtype = "int4"
    with pytest.raises(ValueError):
        model_dtype(cfg, "cpu")
    cfg.model.dtype = "bf16"
    cfg.model.image_model = "solid"
    svc = build_service(cfg)
    gens = {id(r.image_gen) for r in svc.rooms.values()}
    assert len(gens) == 1                               # one shared, batched pipeline
    g = next(iter(svc.rooms.values())).image_gen
    assert isinstance(g, BatchingImageGenerator) and g.max_batch == 2 and g.window_s > 0
    assert not hasattr(cfg.model, "images_per_room")


def test_store_is_thread_safe_under_concurrent_expiry():
    clock = FakeClock()
    st = StateStore(clock)
    errors = []

    def writer(k):
        try:
            for i in range(3000):
                st.hset(f"h{k}", mapping={"a": i, "b": i})
                st.expire(f"h{k}", 0.001 if i % 7 == 0 else 100)
                st.sadd("s", f"{k}:{i % 50}")
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    def reader():
        try:
            for _ in range(3000):
                clock._t += 0.0005             # time moves under the writers
                for k in range(4):
                    st.hgetall(f"h{k}")
                    st.exists(f"h{k}")
                st.scard("s")
                st.snapshot()
        except Exception as e:  # noqa: BLE001
            errors.append(e)
    ths = [threading.Thread(target=writer, args=(k,)) for k in range(4)] + [threading.Thread(target=reader)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=60)
    assert not errors, errors[:3]


def test_tracer_defers_polling_during_capture():
    from cassmantle_amd.utils.tracing import Tracer

    class Ev:
        queried = 0

        def query(self):
            Ev.queried += 1
            return True

        def elapsed_time(self, other):
            return 1.0
    tr = Tracer()
    tr._pending.append(("denoise", Ev(), Ev()))
    with tr.capturing():
        assert tr.poll() == 0 and Ev.queried == 0         # no event query while capturing
    assert tr.poll() == 1 and Ev.queried == 1
