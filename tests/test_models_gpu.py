"""Model-level parity on the GPU: the fused-HIP-kernel models against the same random-init
weights run through plain PyTorch ops (fp32 reference on CPU, or stock ops on the GPU)."""
import math
import pytest
import torch

pytestmark = pytest.mark.gpu

from cassmantle_amd import ops  # noqa: E402


def cos(a, b):
    a = a.float().flatten()
    b = b.float().flatten()
    return (a @ b / (a.norm() * b.norm())).item()


def test_tiny_unet_matches_cpu_reference():
    from cassmantle_amd.models.unet import TINY_UNET, UNet
    m = UNet(TINY_UNET, seed=3)
    x = torch.randn(2, 8, 8, 4).to(torch.bfloat16)
    t = torch.tensor([10.0, 500.0])
    ctx = torch.randn(2, 77, 32).to(torch.bfloat16)
    ref = m(x, t, ctx)
    mg = m.to("cuda")
    out = mg(x.cuda(), t.cuda(), ctx.cuda())
    assert cos(out.cpu(), ref) > 0.995


def test_sd15_unet_hip_vs_stock_torch():
    from cassmantle_amd.models.unet import SD15_UNET, UNet
    m = UNet(SD15_UNET, seed=0).cuda()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 64, 64, 4, generator=g).to(torch.bfloat16).cuda()
    t = torch.tensor([981.0, 981.0], device="cuda")
    ctx = torch.randn(2, 77, 768, generator=g).to(torch.bfloat16).cuda()
    with torch.no_grad():
        out = m(x, t, ctx)
        ops.set_mode("torch")
        try:
            exp = m(x, t, ctx)
        finally:
            ops.set_mode("hip")
    assert torch.isfinite(out.float()).all()
    assert cos(out, exp) > 0.99


def test_vae_and_text_encoders_hip_vs_cpu():
    from cassmantle_amd.models.text import TINY_BERT, TINY_CLIP, CLIPTextEncoder, MiniLMEncoder
    from cassmantle_amd.models.vae import TINY_VAE, VAEDecoder
    vae = VAEDecoder(TINY_VAE, seed=1)
    z = torch.randn(1, 8, 8, 4).to(torch.bfloat16)
    ref = vae(z)
    out = vae.cuda()(z.cuda())
    assert cos(out.cpu(), ref) > 0.995
    clip = CLIPTextEncoder(TINY_CLIP, seed=2)
    ids, _ = clip.tokenizer(["a red fox", "negative"], pad_to=77)
    ref, _ = clip(ids)
    out, _ = clip.cuda()(ids.cuda())
    assert cos(out.cpu(), ref) > 0.995
    bert = MiniLMEncoder(TINY_BERT, seed=3)
    ids, lens = bert.tokenizer(["lantern", "the glowing river bank"], pad_to=16)
    ref = bert(ids, lens)
    out = bert.cuda()(ids.cuda(), lens.cuda())
    assert cos(out.cpu(), ref) > 0.995


def test_pipeline_graph_replay_matches_eager():
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.models.schedulers import make_plan
    sd_g = StableDiffusion(SPECS["tiny"], device="cuda", use_graphs=True, seed=5)
    sd_e = StableDiffusion(SPECS["tiny"], device="cuda", use_graphs=False, seed=5)
    plan = make_plan("pndm", 6, 7.5)
    ctx, _ = sd_e.encode_prompt(["a castle"], "blurry")
    x0 = sd_e.init_latents([7], plan)
    a = sd_e.denoise(ctx, x0, plan).clone()
    b = sd_g.denoise(ctx, x0, plan).clone()
    c = sd_g.denoise(ctx, x0, plan).clone()   # second replay of the same graph
    assert torch.allclose(a, b, atol=1e-3, rtol=1e-3)
    assert torch.allclose(b, c)


def _fp32_cpu_copy(m):
    import copy
    c = copy.deepcopy(m).float().cpu()
    return c


def test_sd15_unet_full_size_vs_fp32_reference():
    """ONE full SD-1.5 UNet evaluation (batch 1, 64^2 latent, 77-token context) on the HIP
    kernels vs the same weights through the fp32 PyTorch reference ops on the CPU"""
    from cassmantle_amd.models.unet import SD15_UNET, UNet
    m = UNet(SD15_UNET, seed=0).cuda()
    g = torch.Generator().manual_seed(0)
    x = torch.randn(1, 64, 64, 4, generator=g).to(torch.bfloat16)
    t = torch.tensor([601.0])
    ctx = (torch.randn(1, 77, 768, generator=g) * 0.5).to(torch.bfloat16)
    with torch.no_grad():
        out = m(x.cuda(), t.cuda(), ctx.cuda()).float().cpu()
        ref = _fp32_cpu_copy(m)(x.float(), t, ctx.float())
    assert torch.isfinite(out).all()
    c = cos(out, ref)
    assert c >= 0.999, c


def test_sd15_unet_bench_batch8_plans():
    """The headline bench's UNet shape: batch 8 (4 images x CFG) at 64^2, i.e. the M = 32768 /
    8192 / 2048 / 512 GEMM rows with the tuned split-K and producer-wave plans the bench runs.
    Every row against the fp32 CPU reference (cos >= 0.999), and against batch-2 runs of the same
    inputs, which take other plans: the two agree to cos >= 0.9998 (bf16 rounding of different
    reduction orders) and the batch-8 rows are no further from fp32 than the batch-2 rows."""
    from cassmantle_amd.models.unet import SD15_UNET, UNet
    m = UNet(SD15_UNET, seed=0).cuda()
    g = torch.Generator().manual_seed(11)
    x = torch.randn(8, 64, 64, 4, generator=g).to(torch.bfloat16)
    t = torch.tensor([801.0] * 8)
    ctx = (torch.randn(8, 77, 768, generator=g) * 0.5).to(torch.bfloat16)
    with torch.no_grad():
        out8 = m(x.cuda(), t.cuda(), ctx.cuda()).float().cpu()
        assert torch.isfinite(out8).all()
        out2 = torch.cat([m(x[i:i + 2].cuda(), t[i:i + 2].cuda(), ctx[i:i + 2].cuda()).float().cpu()
                          for i in range(0, 8, 2)])
        cpu = _fp32_cpu_copy(m)
        ref = torch.cat([cpu(x[i:i + 2].float(), t[i:i + 2], ctx[i:i + 2].float()) for i in range(0, 8, 2)])
    c8 = [cos(out8[r], ref[r]) for r in range(8)]
    c2 = [cos(out2[r], ref[r]) for r in range(8)]
    c82 = [cos(out8[r], out2[r]) for r in range(8)]
    print("cos(b8, fp32)", c8, "cos(b2, fp32)", c2, "cos(b8, b2)", c82)
    assert min(c8) >= 0.999, c8
    assert min(c82) >= 0.9998, c82
    assert min(a - b for a, b in zip(c8, c2)) >= -1e-4, (c8, c2)


def test_sd_vae_decoder_full_size_vs_fp32_reference():
    """the full SD VAE decoder (64^2 latent -> 512^2 image: 512-channel convs, the d=512
    mid-block attention, the parity upsampling convs) vs the fp32 reference"""
    from cassmantle_amd.models.vae import SD_VAE, VAEDecoder
    vae = VAEDecoder(SD_VAE, seed=1).cuda()
    z = torch.randn(1, 64, 64, 4, generator=torch.Generator().manual_seed(3)).to(torch.bfloat16)
    with torch.no_grad():
        out = vae(z.cuda()).float().cpu()
        ref = _fp32_cpu_copy(vae)(z.float())
    assert out.shape == ref.shape == (1, 512, 512, 3)
    c = cos(out, ref)
    assert c >= 0.999, c


@pytest.mark.parametrize("fp8", [False, True])
def test_sdxl_unet_reduced_depth_full_width(fp8):
    """SDXL UNet widths (320/640/1280, head dim 64, 2048-d context, add-embeds) at reduced
    transformer depth and a 32^2 latent, bf16 and OCP-fp8 attention, vs the fp32 reference"""
    import dataclasses
    from cassmantle_amd.models.unet import SDXL_UNET, UNet
    cfg = dataclasses.replace(SDXL_UNET, transformer_depth=(0, 1, 1), mid_transformer_depth=1, sample_size=32)
    m = UNet(cfg, seed=4).cuda()
    g = torch.Generator().manual_seed(5)
    x = torch.randn(1, 32, 32, 4, generator=g).to(torch.bfloat16)
    t = torch.tensor([500.0])
    ctx = (torch.randn(1, 77, 2048, generator=g) * 0.5).to(torch.bfloat16)
    added = {"time_ids": torch.tensor([[256.0, 256.0, 0.0, 0.0, 256.0, 256.0]]),
             "text_embeds": (torch.randn(1, 1280, generator=g) * 0.5).to(torch.bfloat16)}
    with torch.no_grad():
        out = m(x.cuda(), t.cuda(), ctx.cuda(), {k: v.cuda() for k, v in added.items()}, fp8=fp8).float().cpu()
        ref = _fp32_cpu_copy(m)(x.float(), t, ctx.float(), {k: v.float() for k, v in added.items()})
    c = cos(out, ref)
    assert c >= (0.995 if fp8 else 0.999), c


@pytest.mark.parametrize("fp8", [False, True])
def test_sdxl_chained_ln_row_stats_match_stats_pass(fp8):
    """SDXL transformer stacks deeper than one block at >= 1024 rows (the 32^2 level of a 1024^2
    image): block i's feed-forward output projection accumulates the row statistics of its
    output for block i + 1's folded LayerNorm (unet._FF_ROWSTATS) -- same UNet output as the
    row-statistics pass it replaces"""
    import dataclasses
    import cassmantle_amd.models.unet as U
    cfg = dataclasses.replace(U.SDXL_UNET, transformer_depth=(0, 1, 3), mid_transformer_depth=2, sample_size=128)
    m = U.UNet(cfg, seed=4).cuda()
    g = torch.Generator().manual_seed(6)
    x = torch.randn(1, 128, 128, 4, generator=g).to(torch.bfloat16).cuda()
    t = torch.tensor([500.0]).cuda()
    ctx = (torch.randn(1, 77, 2048, generator=g) * 0.5).to(torch.bfloat16).cuda()
    added = {"time_ids": torch.tensor([[1024.0, 1024.0, 0.0, 0.0, 1024.0, 1024.0]]).cuda(),
             "text_embeds": (torch.randn(1, 1280, generator=g) * 0.5).to(torch.bfloat16).cuda()}
    old = U._FF_ROWSTATS
    with torch.no_grad():
        try:
            U._FF_ROWSTATS = True
            a = m(x, t, ctx, added, fp8=fp8).float()
            U._FF_ROWSTATS = False
            b = m(x, t, ctx, added, fp8=fp8).float()
        finally:
            U._FF_ROWSTATS = old
    assert torch.isfinite(a).all()
    c = cos(a.cpu(), b.cpu())
    assert c >= 0.9999, c


def test_fp8_cross_kv_survives_batch_size_change_under_graphs():
    """the e4m3 cross-attention K/V image must be kept per context shape.  A
    graph captured at B=1, then a generation at B=2, then a replay at B=1 must give exactly the
    first B=1 image (the B=1 graph keeps reading its own, refilled, K/V image) and match eager."""
    import dataclasses
    from cassmantle_amd.models.schedulers import make_plan  # noqa: F401
    from cassmantle_amd.models.unet import TINY_UNET
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    unet = dataclasses.replace(TINY_UNET, block_out_channels=(64, 128), heads=(1, 2), head_dim=64,
                               cross_attention_dim=32)
    spec = dataclasses.replace(SPECS["tiny"], name="tiny64", unet=unet)
    g = StableDiffusion(spec, device="cuda", use_graphs=True, fp8_attention=True, seed=7)
    e = StableDiffusion(spec, device="cuda", use_graphs=False, fp8_attention=True, seed=7)
    p1, p2 = ["a lantern"], ["an ember", "a tower"]
    a = g.generate_tensor(p1, "blurry", [3], steps=4).clone()
    lat_a = g.last_latents.float().clone()
    g.generate_tensor(p2, "blurry", [4, 5], steps=4)
    torch.cuda.synchronize()
    c = g.generate_tensor(p1, "blurry", [3], steps=4).clone()
    lat_c = g.last_latents.float().clone()
    e.generate_tensor(p1, "blurry", [3], steps=4)
    lat_e = e.last_latents.float().clone()
    torch.cuda.synchronize()
    assert torch.equal(a, c)
    assert torch.equal(lat_a, lat_c)
    assert torch.allclose(lat_a, lat_e, atol=2e-2, rtol=2e-2), (lat_a - lat_e).abs().max()


def test_sd15_end_to_end_graph_vs_fp32_reference():
    """a whole 4-step generation (CLIP encode -> graph-replayed denoise -> VAE decode -> uint8)
    vs the same pipeline on the fp32 reference path: the images must agree, not just the shape"""
    import numpy as np
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    sd = StableDiffusion(SPECS["sd15"], device="cuda", use_graphs=True, seed=0)
    prompt = ["A cubism style piece depicting the following: a lantern"]
    img = sd.generate(prompt, "blurry", [1], steps=4)[0]
    ref_sd = StableDiffusion(SPECS["sd15"], device="cpu", use_graphs=False, seed=0, dtype=torch.float32)
    with torch.no_grad():                    # identical (bf16-valued) weights, fp32 arithmetic
        for a, b in [(sd.unet, ref_sd.unet), (sd.vae, ref_sd.vae)] + list(zip(sd.text_encoders, ref_sd.text_encoders)):
            b.load_state_dict({k: v.float().cpu() for k, v in a.state_dict().items()})
        ref_sd.unet.fuse_projections()
    ref = ref_sd.generate(prompt, "blurry", [1], steps=4)[0]
    assert img.shape == ref.shape == (512, 512, 3) and img.dtype == np.uint8
    d = np.abs(img.astype(np.float32) - ref.astype(np.float32))
    psnr = 10 * np.log10(255.0 ** 2 / max(float((d ** 2).mean()), 1e-9))
    print(f"[e2e] psnr {psnr:.2f} dB, mean |diff| {d.mean():.3f}")
    # measured 42.7 dB (round 2); 38 dB leaves ~5 dB for kernel-order rounding changes
    assert psnr >= 38.0 and d.mean() < 2.0, (psnr, d.mean())


def test_unet_is_bit_deterministic_run_to_run():
    """The fused GroupNorm statistics use exact integer (fixed-point) atomics, so two evaluations
    of the same inputs are bit-identical (fp32 atomics made them differ at the bf16 level)."""
    from cassmantle_amd.models.unet import SD15_UNET, UNet
    m = UNet(SD15_UNET, seed=1).cuda()
    g = torch.Generator().manual_seed(2)
    x = torch.randn(8, 32, 32, 4, generator=g).to(torch.bfloat16).cuda()
    t = torch.full((8,), 700.0, device="cuda")
    ctx = torch.randn(8, 77, 768, generator=g).to(torch.bfloat16).cuda()
    with torch.no_grad():
        a = m(x, t, ctx)
        b = m(x, t, ctx)
    assert torch.equal(a, b)


def test_legacy_stream_scorer_not_blocked_by_generation():
    """the round-1 'stall': a scorer on the thread's LEGACY default stream while another thread
    generates.  generate() must not enqueue anything on the legacy stream, so scoring keeps its
    latency while a generation is in flight (it queued behind whole generations before)."""
    import threading
    import time
    import numpy as np
    from cassmantle_amd.game.scoring import score_pairs
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    from cassmantle_amd.scoring.encoder import EncoderBackend
    sd = StableDiffusion(SPECS["sd15"], device="cuda", seed=0)
    sd.generate(["a lantern"] * 2, "blurry", [0, 1], steps=4)          # capture
    be = EncoderBackend(device="cuda", use_graphs=False)
    be.stream = None                                                    # legacy default stream
    pairs = [(w, "tower") for w in ("lantern", "river", "ember", "shadow")]
    score_pairs(be, pairs, 0.01)
    stop = threading.Event()
    gens = [0]

    def loop():
        while not stop.is_set():
            sd.generate(["a lantern"] * 2, "blurry", [2, 3], steps=12)
            gens[0] += 1
    th = threading.Thread(target=loop, daemon=True)
    th.start()
    time.sleep(0.5)
    lat = []
    t_end = time.perf_counter() + 6.0
    while time.perf_counter() < t_end:
        t0 = time.perf_counter()
        score_pairs(be, pairs, 0.01)
        lat.append((time.perf_counter() - t0) * 1e3)
    stop.set()
    th.join(timeout=60)
    assert gens[0] >= 1
    # one 12-step generation of 2 images takes ~100 ms: queueing behind it would put p50 there
    assert len(lat) > 100 and float(np.percentile(lat, 50)) < 20.0, (len(lat), np.percentile(lat, 50))
    print(f"[legacy-stream scorer] {len(lat)} calls, p50 {np.percentile(lat, 50):.2f} ms, p90 {np.percentile(lat, 90):.2f} ms")


def test_stage_overlap_decode_matches_serial():
    """stage overlap: generation i's VAE decode runs on the decode stream while generation i+1
    denoises; back-to-back un-synchronised calls must still give exactly the serial images"""
    from cassmantle_amd.pipeline import SPECS, StableDiffusion
    a = StableDiffusion(SPECS["sd15"], device="cuda", seed=0, overlap_decode=True)
    b = StableDiffusion(SPECS["sd15"], device="cuda", seed=0, overlap_decode=False)
    prompts = [["a lantern", "a river"], ["an ember", "a tower"], ["a shadow", "a forest"]]
    outs = [a.generate_tensor(p, "blurry", [i, i + 10], steps=6, sync_caller=False) for i, p in enumerate(prompts)]
    torch.cuda.synchronize()
    ref = [b.generate_tensor(p, "blurry", [i, i + 10], steps=6) for i, p in enumerate(prompts)]
    torch.cuda.synchronize()
    for x, y in zip(outs, ref):
        assert torch.equal(x, y)


def test_clip_encode_graph_matches_eager():
    """the graph-captured text encoder (one capture per batch shape, replayed per generation)
    gives the eager encoder's output, and a second replay with other prompts is not stale"""
    from cassmantle_amd.models.text import CLIP_L, CLIPTextEncoder
    enc = CLIPTextEncoder(CLIP_L, seed=2).cuda()
    with torch.no_grad():
        for texts in (["a lantern by the river", "blurry"], ["an ember in the tower", "fake, abstract"]):
            h_e, _ = enc.encode(texts, "cuda", output_hidden=-2)
            h_g, _ = enc.encode(texts, "cuda", output_hidden=-2, graphs=True)
            torch.cuda.synchronize()
            assert torch.equal(h_e, h_g)
