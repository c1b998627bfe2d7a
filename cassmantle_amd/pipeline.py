"""On-device txt2img pipeline (SD-1.5 / SDXL) with a hipGraph-captured denoise step.

Replaces the reference's remote ``generate_image`` call (``src/backend.py:270-295``; the HF
endpoint ran CLIP encode → UNet denoise loop → VAE decode remotely).  The denoise loop is the
hot loop of the whole framework, so:

* all step-dependent inputs (UNet timestep, scheduler coefficients, multistep history) live
  in device buffers indexed by a device step counter; one step = UNet forward (CFG batch 2B)
  + the fused latent-step kernel + a counter bump, with no host synchronisation;
* that step is captured ONCE per (batch, resolution, scheduler) as a ``torch.cuda.CUDAGraph``
  (a hipGraph on ROCm) and replayed ``evals`` times, removing the ~400 per-step launches' host
  cost;
* text encoding, latents and VAE decode use the same fused-op model code.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import ops
from .game.content import ImageGenerator, ImageGenerationError
from .models.schedulers import SchedulePlan, make_plan
from .models.text import CLIP_BIGG, CLIP_L, TINY_CLIP, CLIPTextEncoder, CLIPTextConfig
from .models.unet import SD15_UNET, SDXL_UNET, TINY_UNET, UNet, UNetConfig
from .models.vae import SD_VAE, SDXL_VAE, TINY_VAE, VAEConfig, VAEDecoder
from .utils.tracing import TRACER, span


@dataclass
class PipelineSpec:
    name: str
    unet: UNetConfig
    vae: VAEConfig
    text: Tuple[CLIPTextConfig, ...]
    resolution: int
    steps: int
    scheduler: str
    guidance: float = 7.5


SPECS: Dict[str, PipelineSpec] = {
    "sd15": PipelineSpec("sd15", SD15_UNET, SD_VAE, (CLIP_L,), 512, 50, "pndm"),
    "sdxl": PipelineSpec("sdxl", SDXL_UNET, SDXL_VAE, (CLIP_L, CLIP_BIGG), 1024, 30, "euler", 5.0),
    "tiny": PipelineSpec("tiny", TINY_UNET, TINY_VAE, (TINY_CLIP,), 16, 4, "ddim"),
}


def default_device() -> torch.device:
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


# VAE decode captured as a graph per step state: OFF by default -- measured slower than the eager
# decode (13.5 vs 11.1 ms per 4-image decode, 558-560 vs 557-558 ms/step, same box x2,
# profiles/r3_vae_graph_ab.txt); CASSMANTLE_VAE_GRAPH=1 turns it on
_VAE_GRAPH = os.environ.get("CASSMANTLE_VAE_GRAPH", "0") == "1"
# text encoders captured as a graph per batch shape (CLIPTextEncoder.encode(graphs=True));
# opt-in (CASSMANTLE_TEXT_GRAPH=1): no measured gain (profiles/r3_fusions_ab.txt)
_TEXT_GRAPH = os.environ.get("CASSMANTLE_TEXT_GRAPH", "0") == "1"
# (The CFG batch as concurrent row-range branches on parallel streams inside the captured step was
# measured 7-13 % slower than one batch-8 stream, profiles/r3_unet_branches_ab.txt; removed in
# round 4, kept in git history.)


class _StepState:
    """Static device buffers of one denoise configuration (graph-capture friendly)."""

    def __init__(self, B: int, h: int, w: int, ctx: torch.Tensor, plan: SchedulePlan, device, dtype,
                 cfg: bool, added: Optional[dict]):
        self.B, self.cfg = B, cfg
        nb = 2 * B if cfg else B
        # (latent_init fills x / xs / hist at every load; zero fills on the GPU are HIP kernels)
        self.x = torch.empty((B, h, w, 4), device=device, dtype=torch.float32)
        self.xs = torch.empty_like(self.x)
        self.hist = torch.empty((4, B, h, w, 4), device=device, dtype=torch.float32)
        # on the GPU the UNet input carries 4 zero channels: conv_in then reads whole 16-byte
        # k-chunks with no per-step pad copy (the latent-step kernel writes channels 0..3)
        self.unet_in = ops.zero_(torch.empty((nb, h, w, 8 if torch.device(device).type == "cuda" else 4),
                                             device=device, dtype=dtype))
        self.ctx = torch.empty_like(ctx)
        self.coef = torch.from_numpy(plan.table).to(device)
        self.tsteps = torch.from_numpy(plan.table[:, 14].copy()).to(device)
        # the time table's per-row inputs, built on the host once per state: t of row e*nb + b
        # and the row -> image index of the add-embedding repeat (no device repeat kernels)
        E = plan.table.shape[0]
        self.t_rep = torch.from_numpy(np.repeat(plan.table[:, 14].astype(np.float32), nb)).to(device)
        self.rep_ids = torch.from_numpy((np.arange(E * nb) % nb).astype(np.int32)).to(device)
        self.tid_rep = None
        if added is not None:
            self.tid_rep = added["time_ids"].detach().cpu().repeat(E, 1).to(device)
        self.z = torch.empty((B, h, w, 4), device=device, dtype=dtype)      # bf16 latents for the VAE
        self.finite = torch.empty((16,), device=device, dtype=torch.uint8)[:1]   # set by finalize_latents
        self.step = ops.zero_(torch.empty((4,), device=device, dtype=torch.int32))[:1]
        self.added = None
        if added is not None:
            self.added = {k: torch.empty_like(v) for k, v in added.items()}
        self.graph: Optional["torch.cuda.CUDAGraph"] = None
        # captured VAE decode of ``z`` and its static uint8 output (StableDiffusion._decode)
        self.vae_graph: Optional["torch.cuda.CUDAGraph"] = None
        self.vae_img: Optional[torch.Tensor] = None
        self.plan = plan
        # per-plan time conditioning (UNet.time_table), refilled in place every generation
        self.temb_tab: Optional[torch.Tensor] = None
        self.tb_tab: Optional[torch.Tensor] = None
        # the current step's rows, refilled by the latent-step launch for the next step
        self.temb_cur: Optional[torch.Tensor] = None
        self.tb_cur: Optional[torch.Tensor] = None

    def load_time(self, temb: torch.Tensor, tb: torch.Tensor) -> None:
        if self.temb_tab is None:
            self.temb_tab, self.tb_tab = temb.clone(), tb.clone()
            self.temb_cur, self.tb_cur = temb[0].clone(), tb[0].clone()
        else:
            ops.copy_(self.temb_tab, temb)
            ops.copy_(self.tb_tab, tb)

    def load(self, x0: torch.Tensor, ctx: torch.Tensor, added: Optional[dict]):
        # x, xs, hist and the first UNet input (both CFG halves) in one kernel
        ops.latent_init(x0, self.plan.c_in0, self.x, self.xs, self.hist, self.unet_in, self.cfg)
        # (in-tree copy kernels: no runtime blit in a generation's trace)
        ops.copy_(self.ctx, ctx)
        if self.temb_tab is not None:
            ops.copy_(self.temb_cur, self.temb_tab[0])
            ops.copy_(self.tb_cur, self.tb_tab[0])
        if added is not None:
            for k, v in added.items():
                ops.copy_(self.added[k], v)
        ops.zero_(self.step)


class StableDiffusion:
    def __init__(self, spec: PipelineSpec, device=None, dtype=torch.bfloat16, seed: int = 0,
                 use_graphs: bool = True, fp8_attention: bool = False, overlap_decode: bool = False,
                 stream: Optional["torch.cuda.Stream"] = None) -> None:
        self.spec = spec
        self.device = torch.device(device) if device is not None else default_device()
        self.dtype = dtype
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self.fp8 = fp8_attention
        self.text_encoders = [CLIPTextEncoder(c, seed=seed + i, dtype=dtype).to(self.device).eval()
                              for i, c in enumerate(spec.text)]
        # derived weights (fused projections, LayerNorm folds, parity-folded upsampling convs,
        # padded conv_in, scaled post-quant conv) are computed on the CPU BEFORE the move: no
        # setup kernel of ATen / hipBLASLt / rocBLAS runs on the GPU (verdict r2 item 7)
        self.unet = UNet(spec.unet, seed=seed, dtype=dtype).prepare().to(self.device).eval()
        self.vae = VAEDecoder(spec.vae, seed=seed, dtype=dtype).prepare().to(self.device).eval()
        self._states: Dict[tuple, _StepState] = {}
        self.timings: Dict[str, float] = {}
        # generation runs on its own stream (never the legacy default stream), so a serving
        # process can overlap it with the scorer's high-priority stream (BASELINE config 5)
        # (``stream``: a caller-made stream, e.g. CU-masked by runtime.cumask so the serving
        # scorer keeps a few CUs of its own)
        self.stream = stream if stream is not None else (
            torch.cuda.Stream(device=self.device) if self.device.type == "cuda" else None)
        # stage overlap (opt-in): the VAE decode of generation i runs on its own stream,
        # concurrently with the encode + denoise of generation i+1 (the latents it reads are a
        # bf16 copy, so the next denoise may overwrite the step state at once).  Measured OFF by
        # default: 605 vs 599 ms per 4-image step on MI355X, same box interleaved x2
        # (profiles/r2_stage_overlap_ab.txt) -- the decode's kernels slow the concurrent graph
        # replay by more than the 21 ms of encode + decode they hide
        self.decode_stream = (torch.cuda.Stream(device=self.device)
                              if self.device.type == "cuda" and overlap_decode else None)
        # one generation at a time per pipeline: the per-shape step state (latents, K/V context
        # buffers, time table, captured graph) is shared, so concurrent callers (several rooms'
        # worker threads) must not interleave (serving batches rooms through
        # BatchingImageGenerator instead of queueing on this lock)
        self._lock = threading.RLock()
        # device flag: were the final latents of the last generation finite (checked before the
        # uint8 decode, where NaN/Inf would silently become a garbage image)
        self.last_finite: Optional[torch.Tensor] = None

    @property
    def latent_size(self) -> int:
        return self.spec.resolution // (2 ** (len(self.spec.vae.block_out_channels) - 1))

    # ------------------------------------------------------------------ text
    @torch.no_grad()
    def encode_prompt(self, prompts: Sequence[str], negative: str) -> Tuple[torch.Tensor, Optional[dict]]:
        """-> ctx [2B, 77, D] ordered (uncond..., cond...), optional SDXL add-embeds."""
        texts = [negative] * len(prompts) + list(prompts)
        if len(self.text_encoders) == 1:
            ctx, _ = self.text_encoders[0].encode(texts, self.device, graphs=self.use_graphs and _TEXT_GRAPH)
            return ctx, None
        hs, pooled = [], None
        for enc in self.text_encoders:
            h, p = enc.encode(texts, self.device, output_hidden=-2, graphs=self.use_graphs and _TEXT_GRAPH)
            hs.append(h)
            if p is not None:
                pooled = p
        ctx = ops.concat_last(hs[0], hs[1]) if len(hs) == 2 else torch.cat(hs, dim=-1)
        R = self.spec.resolution
        tid = ops.h2d(torch.tensor([R, R, 0, 0, R, R], dtype=torch.float32).repeat(len(texts), 1), self.device)
        return ctx, {"time_ids": tid, "text_embeds": pooled}

    # ------------------------------------------------------------------ denoise
    def _unet_step(self, st: _StepState) -> None:
        # this step's rows of the per-plan time tables (st.*_cur: filled for step 0 by load(),
        # then by the previous step's latent-step launch from the device step counter)
        eps = self.unet(st.unet_in, None, st.ctx, st.added, fp8=self.fp8, time_cond=(st.temb_cur, st.tb_cur))
        ops.latent_step(eps, st.x, st.hist, st.xs, st.coef, st.step, st.unet_in, st.cfg,
                        rows=[(st.temb_tab, st.temb_cur), (st.tb_tab, st.tb_cur)])
        ops.advance_step(st.step)

    def prepare(self) -> None:
        """Recompute the derived weights (after an in-place weight load).  Captured step / decode
        graphs point at the old derived buffers, so the per-shape states are dropped (recaptured
        on the next generation)."""
        with self._lock:
            self.unet.prepare()
            self.vae.prepare()
            self._states.clear()

    def _state(self, B: int, ctx: torch.Tensor, plan: SchedulePlan, added) -> _StepState:
        key = (B, self.latent_size, plan.name, plan.evals, float(plan.table[0, 13]), tuple(ctx.shape))
        st = self._states.get(key)
        if st is None:
            h = w = self.latent_size
            st = _StepState(B, h, w, ctx, plan, self.device, self.dtype, cfg=True, added=added)
            self._states[key] = st
        return st

    def _capture(self, st: _StepState) -> None:
        # warm up on a side stream (allocator / kernel autotune), then capture one step
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._unet_step(st)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        # thread_local capture mode: other threads (the scorer's stream, a metrics scrape) may
        # keep making CUDA calls while this thread captures; the tracer also defers its event
        # queries for the duration
        with TRACER.capturing(), torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._unet_step(st)
        st.graph = g

    def _decode(self, st: _StepState, z: torch.Tensor) -> torch.Tensor:
        """VAE decode -> uint8 image.  With graphs, the decode of the state's latent buffer is
        captured once per state and replayed (~200 eager launches per generation otherwise: host
        time that also holds the GIL against a serving process's scorer thread); the replay's
        static output is copied out, so the returned image outlives the next generation."""
        if not self.use_graphs or not _VAE_GRAPH or z is not st.z:
            return self.vae.decode_uint8(z)
        if st.vae_graph is None:
            s = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                self.vae.decode_uint8(z)                       # warm-up: allocator, tuning tables
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with TRACER.capturing(), torch.cuda.graph(g, capture_error_mode="thread_local"):
                st.vae_img = self.vae.decode_uint8(z)
            st.vae_graph = g
        st.vae_graph.replay()
        out = torch.empty_like(st.vae_img)
        ops.copy_(out, st.vae_img)
        return out

    @torch.no_grad()
    def denoise(self, ctx: torch.Tensor, latents: torch.Tensor, plan: SchedulePlan,
                added: Optional[dict] = None) -> torch.Tensor:
        B = latents.shape[0]
        st = self._state(B, ctx, plan, added)
        self._last_state = st
        # cross-attention K/V of the (loop-invariant) text context: one GEMM per generation,
        # written into per-shape buffers that the captured step graph reads
        self.unet.set_context(ctx, fp8=self.fp8)
        # time embedding + every ResNet's time bias for all timesteps of the plan: one batched
        # MLP + GEMM per generation (in place, so a captured step graph reads the new values)
        added_t = dict(added, time_ids_rep=st.tid_rep) if added is not None and st.tid_rep is not None else added
        st.load_time(*self.unet.time_table(st.tsteps, st.unet_in.shape[0], added_t, t_rep=st.t_rep,
                                           rep_ids=st.rep_ids))
        if self.use_graphs and st.graph is None:
            st.load(latents, ctx, added)
            self._capture(st)
        st.load(latents, ctx, added)
        for _ in range(plan.evals):
            if st.graph is not None:
                st.graph.replay()
            else:
                self._unet_step(st)
        return st.x

    # ------------------------------------------------------------------ full pipeline
    def init_latents(self, seeds: Sequence[int], plan: SchedulePlan) -> torch.Tensor:
        h = self.latent_size
        xs = []
        for s in seeds:
            g = torch.Generator().manual_seed(int(s))
            xs.append(torch.randn((h, h, 4), generator=g, dtype=torch.float32))
        return ops.h2d(torch.stack(xs) * plan.init_sigma, self.device)

    @torch.no_grad()
    def generate_tensor(self, prompts: Sequence[str], negative: str, seeds: Sequence[int],
                        steps: Optional[int] = None, guidance: Optional[float] = None,
                        scheduler: Optional[str] = None, sync_caller: bool = True) -> torch.Tensor:
        """-> uint8 [B, H, W, 3] on device.  With ``sync_caller`` the caller's current stream is
        made to wait for the generation (the tensor is then safe to use on it); without it the
        result is ordered only on ``self.stream`` and the caller synchronises that stream.

        Stall root cause (round 1, tools/repro_stall.py, profiles/r2_stall_repro_*.log): a
        thread with no stream of its own has the process-wide LEGACY default stream as its
        current stream.  ``caller.wait_stream(self.stream)`` there inserts a wait for the WHOLE
        denoise loop into that shared stream, so every kernel another thread (the scorer)
        submits to the legacy stream afterwards queues behind the generation: 28 score batches/s
        vs 832/s on its own stream, with generation throughput unchanged.  Serving therefore
        never passes the legacy stream here (``generate`` copies on ``self.stream``), and the
        scorer always owns a non-blocking stream."""
        plan = make_plan(scheduler or self.spec.scheduler, steps or self.spec.steps,
                         self.spec.guidance if guidance is None else guidance)
        with self._lock:
            return self._generate_locked(prompts, negative, seeds, plan, sync_caller)

    def _generate_locked(self, prompts, negative, seeds, plan, sync_caller=True) -> torch.Tensor:
        caller = torch.cuda.current_stream(self.device) if self.stream is not None else None
        with (torch.cuda.stream(self.stream) if self.stream is not None else contextlib.nullcontext()):
            if caller is not None and sync_caller:
                self.stream.wait_stream(caller)     # inputs the caller produced
            # per-stage device time (events on the generation stream: no host sync)
            with span("encode", self.stream):
                ctx, added = self.encode_prompt(prompts, negative)
                x0 = self.init_latents(seeds, plan)
            with span("denoise", self.stream):
                x = self.denoise(ctx, x0, plan, added)
            # bf16 latents for the VAE + finiteness flag of the fp32 latents, one kernel (the
            # flag is checked before the uint8 decode, where NaN/Inf would silently become a
            # garbage image)
            st = self._last_state
            if self.decode_stream is None:
                z, finite = st.z, st.finite
            else:
                # the decode of this generation runs on decode_stream, concurrently with the next
                # generation's finalize_latents on self.stream: fresh buffers per generation, so
                # the next one cannot overwrite the latents (or flag) a running decode reads
                # (record_stream below only keeps the allocator from reusing them)
                z = torch.empty(x.shape, device=x.device, dtype=self.dtype)
                finite = torch.empty((16,), device=x.device, dtype=torch.uint8)[:1]
            ops.finalize_latents(x, z, finite)
            self.last_finite = finite
            self.last_latents = z
            if self.decode_stream is None:
                with span("decode", self.stream):
                    img = self._decode(st, z)
        out_stream = self.stream
        if self.decode_stream is not None:
            self.decode_stream.wait_stream(self.stream)
            with torch.cuda.stream(self.decode_stream), span("decode", self.decode_stream):
                z.record_stream(self.decode_stream)
                self.last_finite.record_stream(self.decode_stream)
                img = self.vae.decode_uint8(z)
            out_stream = self.decode_stream
        self.out_stream = out_stream
        if caller is not None and sync_caller:
            caller.wait_stream(out_stream)
            img.record_stream(caller)
        return img

    def generate(self, prompts: Sequence[str], negative: str, seeds: Sequence[int], **kw) -> List[np.ndarray]:
        with self._lock:
            img = self.generate_tensor(prompts, negative, seeds, sync_caller=False, **kw)
            finite = self.last_finite
            if self.stream is not None:
                # D2H on the stream that produced the image and a wait on THAT stream only:
                # nothing is enqueued on the caller thread's (possibly legacy default) stream
                out = self.out_stream
                with torch.cuda.stream(out):
                    host = torch.empty(img.shape, dtype=img.dtype, pin_memory=True)
                    host.copy_(img, non_blocking=True)
                    ok = torch.empty(finite.shape, dtype=finite.dtype, pin_memory=True)
                    ok.copy_(finite, non_blocking=True)
                out.synchronize()
                arr, fin = host.numpy(), bool(ok.reshape(-1)[0])
            else:
                arr, fin = img.numpy(), bool(finite.reshape(-1)[0])
            if not fin:
                raise ImageGenerationError("non-finite latents (NaN/Inf in the denoise loop)")
        return [arr[i].copy() for i in range(arr.shape[0])]


@dataclass
class DeviceImages:
    """A generation's result left in HBM (multi-GPU data plane, ``parallel.rooms.RankWorker``)."""
    images: torch.Tensor                  # uint8 [B, H, W, 3] on the device
    finite: Optional[torch.Tensor]        # device bool scalar: the final latents were finite
    event: "torch.cuda.Event"             # recorded after the VAE decode on the producing stream


class DiffusionImageGenerator(ImageGenerator):
    """Game-layer adapter (``ImageGenerator``) around :class:`StableDiffusion`."""

    def __init__(self, model: str = "sd15", device=None, steps: Optional[int] = None,
                 guidance: Optional[float] = None, scheduler: Optional[str] = None,
                 use_graphs: bool = True, fp8_attention: bool = False, seed: int = 0,
                 dtype=torch.bfloat16, weights_path: Optional[str] = None, stream=None) -> None:
        self.sd = StableDiffusion(SPECS[model], device=device, use_graphs=use_graphs,
                                  fp8_attention=fp8_attention, seed=seed, dtype=dtype, stream=stream)
        self.weights_loaded: Optional[Dict[str, int]] = None
        if weights_path:
            # diffusers-layout checkpoint (ModelConfig.weights_path); random init otherwise
            from .models.weights import load_pipeline_weights
            self.weights_loaded = load_pipeline_weights(self.sd, weights_path)
        self.resolution = self.sd.spec.resolution
        self.kw = dict(steps=steps, guidance=guidance, scheduler=scheduler)

    def generate(self, prompts, negative_prompt, seeds):
        return self.sd.generate(prompts, negative_prompt, seeds, **self.kw)

    def generate_device(self, prompts, negative_prompt, seeds) -> DeviceImages:
        """``generate`` without the host copy: the images stay on the device, ordered by the
        returned event (the caller's stream waits on it; nothing is enqueued on the caller's
        stream here, see ``StableDiffusion.generate_tensor``)."""
        with self.sd._lock:
            img = self.sd.generate_tensor(prompts, negative_prompt, seeds, sync_caller=False, **self.kw)
            ev = torch.cuda.Event()
            ev.record(self.sd.out_stream)
            return DeviceImages(img, self.sd.last_finite, ev)
