"""CPU tests of the model code on the plain-PyTorch reference ops: shapes, scheduler tables
against independent implementations, checkpoint name/layout mapping round trips, tokenizers."""
import math

import numpy as np
import pytest
import torch

from cassmantle_amd.models import schedulers as S
from cassmantle_amd.models.text import (TINY_BERT, TINY_CLIP, CLIPTextEncoder, MiniLMEncoder,
                                        bert_tokenizer, clip_tokenizer)
from cassmantle_amd.models.unet import TINY_UNET, UNet
from cassmantle_amd.models.vae import TINY_VAE, VAEDecoder
from cassmantle_amd.models.weights import export_diffusers, load_state


def test_tiny_unet_shapes():
    m = UNet(TINY_UNET, seed=1)
    x = torch.randn(2, 8, 8, 4).to(torch.bfloat16)
    out = m(x, torch.tensor([1.0, 999.0]), torch.randn(2, 77, 32).to(torch.bfloat16))
    assert out.shape == (2, 8, 8, 4) and torch.isfinite(out.float()).all()


def test_sd15_unet_parameter_count():
    # SD-1.5 UNet has ~860M parameters [ext]; the fused QKV/KV layout keeps the count
    from cassmantle_amd.models.unet import SD15_UNET
    with torch.device("meta"):
        m = UNet(SD15_UNET, seed=0)
    n = sum(p.numel() for p in m.parameters())
    assert 855e6 < n < 866e6, n


def test_vae_decoder_upsamples():
    v = VAEDecoder(TINY_VAE, seed=0)
    img = v(torch.randn(1, 4, 4, 4).to(torch.bfloat16))
    assert img.shape == (1, 8, 8, 3)


def _ref_pndm(steps, eps_seq, x0):
    """Independent PLMS (skip_prk_steps) re-implementation from the update equations."""
    acp = S.scaled_linear_alphas_cumprod()
    ratio = 1000 // steps
    ts = np.arange(0, steps) * ratio + 1
    plms = list(np.concatenate([ts[:-1], ts[-2:-1], ts[-1:]])[::-1])
    ets, cur, x = [], None, x0.copy()
    for c, t in enumerate(plms):
        e = eps_seq[c]
        prev = t - ratio
        if c != 1:
            ets = ets[-3:] + [e]
        else:
            prev, t = t, t + ratio
        if len(ets) == 1 and c == 0:
            mo, cur = e, x
        elif len(ets) == 1 and c == 1:
            mo, x, cur = (e + ets[-1]) / 2, cur, None
        elif len(ets) == 2:
            mo = (3 * ets[-1] - ets[-2]) / 2
        elif len(ets) == 3:
            mo = (23 * ets[-1] - 16 * ets[-2] + 5 * ets[-3]) / 12
        else:
            mo = (55 * ets[-1] - 59 * ets[-2] + 37 * ets[-3] - 9 * ets[-4]) / 24
        a_t = acp[t]
        a_p = acp[prev] if prev >= 0 else acp[0]
        denom = a_t * (1 - a_p) ** 0.5 + (a_t * (1 - a_t) * a_p) ** 0.5
        x = (a_p / a_t) ** 0.5 * x - (a_p - a_t) * mo / denom
    return x


def _run_table(plan, eps_seq, x0):
    x = torch.from_numpy(x0).float()[None]
    hist = torch.zeros(4, *x.shape)
    xs = torch.zeros_like(x)
    unet_in = torch.zeros_like(x)
    coef = torch.from_numpy(plan.table)
    step = torch.zeros(1, dtype=torch.int32)
    for i in range(plan.evals):
        S.latent_step_reference(torch.from_numpy(eps_seq[i]).float()[None], x, hist, xs, coef, step, unet_in, False)
        step += 1
    return x[0].numpy()


def test_pndm_table_matches_independent_plms():
    steps = 12
    rng = np.random.default_rng(0)
    plan = S.pndm_plan(steps, 7.5)
    assert plan.evals == steps + 1
    eps = [rng.standard_normal(16).astype(np.float64) for _ in range(plan.evals)]
    x0 = rng.standard_normal(16)
    ref = _ref_pndm(steps, eps, x0)
    got = _run_table(plan, [e.astype(np.float32) for e in eps], x0.astype(np.float32))
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-4)


def test_ddim_table_is_deterministic_ddim():
    plan = S.ddim_plan(10, 1.0)
    acp = S.scaled_linear_alphas_cumprod()
    rng = np.random.default_rng(1)
    x0 = rng.standard_normal(8)
    eps = [rng.standard_normal(8) for _ in range(10)]
    x = x0.copy()
    ts = plan.timesteps().astype(int)
    for i, t in enumerate(ts):
        a_t = acp[t]
        a_p = acp[ts[i + 1]] if i + 1 < len(ts) else acp[0]
        x0p = (x - math.sqrt(1 - a_t) * eps[i]) / math.sqrt(a_t)
        x = math.sqrt(a_p) * x0p + math.sqrt(1 - a_p) * eps[i]
    got = _run_table(plan, [e.astype(np.float32) for e in eps], x0.astype(np.float32))
    assert np.allclose(got, x, rtol=1e-4, atol=1e-4)


def test_euler_plan_sigmas():
    plan = S.euler_plan(30, 5.0)
    assert plan.evals == 30 and plan.init_sigma > 10
    assert plan.table[-1, 7] == 1.0 and plan.table[0, 6] < 0


@pytest.mark.parametrize("kind,factory", [
    ("unet", lambda s: UNet(TINY_UNET, seed=s)),
    ("vae", lambda s: VAEDecoder(TINY_VAE, seed=s)),
    ("clip", lambda s: CLIPTextEncoder(TINY_CLIP, seed=s)),
])
def test_checkpoint_roundtrip(kind, factory):
    a, b = factory(1), factory(2)
    sd = export_diffusers(a, kind)
    # on disk every conv kernel is NCHW [Cout, Cin, kh, kw]: it must be exactly our
    # [Cout, kh, kw, Cin] tensor permuted
    own = a.state_dict()
    convs = [n for n, t in own.items() if t.dim() == 4]
    assert convs or kind == "clip"
    for n in convs:
        dn = next(k for k, t in sd.items() if t.dim() == 4 and t.shape == own[n].permute(0, 3, 1, 2).shape
                  and torch.equal(t, own[n].permute(0, 3, 1, 2)))
        assert dn
    if kind == "unet":
        assert any(k.startswith("down_blocks.0.attentions.0.transformer_blocks.0.attn1.to_q") for k in sd)
        assert sd["conv_in.weight"].shape[1] == 4            # NCHW on disk
    missing = load_state(b, sd, kind)
    assert not missing
    for (n1, p1), (n2, p2) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(p1, p2), n1


def test_tokenizers():
    ids, lens = clip_tokenizer()(["a red fox", ""], pad_to=77)
    assert ids.shape == (2, 77) and ids[0, 0] == 49406 and ids[0, 4] == 49407 and ids[1, 1] == 49407
    ids, lens = bert_tokenizer()(["lantern"], pad_to=16)
    assert ids[0, 0] == 101 and ids[0, 2] == 102 and lens[0] == 3


def test_minilm_embeddings_normalised():
    m = MiniLMEncoder(TINY_BERT, seed=0)
    e = m.embed(["lantern", "a glowing river"], "cpu", pad_to=16)
    assert torch.allclose(e.norm(dim=-1), torch.ones(2), atol=1e-4)


def test_time_table_matches_per_step_time_embedding():
    """The sampler's per-plan time table (one batched MLP + GEMM per generation) must give the
    same UNet output as the per-step time embedding, for SD-1.5-style and SDXL-style (add-embeds)
    conditioning."""
    import torch
    from dataclasses import replace
    from cassmantle_amd.models.unet import TINY_UNET, UNet
    for cfg in (TINY_UNET, replace(TINY_UNET, addition_embed=True, addition_time_embed_dim=8,
                                   projection_class_embeddings_input_dim=32 + 6 * 8)):
        m = UNet(cfg, seed=4)
        g = torch.Generator().manual_seed(1)
        x = torch.randn(2, 8, 8, 4, generator=g).to(torch.bfloat16)
        ctx = torch.randn(2, 77, 32, generator=g).to(torch.bfloat16)
        added = None
        if cfg.addition_embed:
            added = {"time_ids": torch.tensor([[16., 16, 0, 0, 16, 16]] * 2),
                     "text_embeds": torch.randn(2, 32, generator=g).to(torch.bfloat16)}
        ts = torch.tensor([999.0, 500.0, 1.0])
        temb, tb = m.time_table(ts, 2, added)
        for e in range(3):
            ref = m(x, ts[e].expand(2), ctx, added)
            out = m(x, None, ctx, added, time_cond=(temb[e], tb[e]))
            assert torch.equal(out, ref)


# ---------------------------------------------------------------- parity with transformers
# Architecture AND checkpoint key mapping pinned against the public implementations (random
# small configs, fp32 on the CPU reference path; the same ids go to both models).

def test_minilm_matches_transformers_bert():
    transformers = pytest.importorskip("transformers")
    from cassmantle_amd.models.text import BertConfig as OurBert, MiniLMEncoder
    from cassmantle_amd.models.weights import export_bert, load_bert
    hf_cfg = transformers.BertConfig(vocab_size=500, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                                     intermediate_size=128, max_position_embeddings=64, hidden_act="gelu",
                                     layer_norm_eps=1e-12, hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    torch.manual_seed(0)
    hf = transformers.BertModel(hf_cfg, add_pooling_layer=False).eval()
    ours = MiniLMEncoder(OurBert(vocab_size=500, max_positions=64, dim=64, layers=2, heads=4, mlp=128),
                         dtype=torch.float32).eval()
    missing = load_bert(ours, hf.state_dict())
    assert not missing
    g = torch.Generator().manual_seed(1)
    ids = torch.randint(1, 500, (3, 12), generator=g)
    lens = torch.tensor([12, 7, 3], dtype=torch.int32)
    mask = (torch.arange(12)[None] < lens[:, None]).long()
    ids = ids * mask
    with torch.no_grad():
        h = hf(input_ids=ids, attention_mask=mask).last_hidden_state
        pooled = (h * mask[..., None]).sum(1) / mask.sum(1, keepdim=True)
        ref = torch.nn.functional.normalize(pooled, dim=-1)
        out = ours(ids, lens)
    assert (out - ref).abs().max().item() < 1e-4
    # the exporter is the inverse mapping
    sd = export_bert(ours)
    assert set(sd) <= set(hf.state_dict()) and all(torch.equal(sd[k], hf.state_dict()[k]) for k in sd)


def test_clip_text_matches_transformers():
    transformers = pytest.importorskip("transformers")
    from cassmantle_amd.models.text import CLIPTextConfig as OurClip
    hf_cfg = transformers.CLIPTextConfig(vocab_size=500, hidden_size=64, intermediate_size=128, num_hidden_layers=2,
                                         num_attention_heads=4, max_position_embeddings=77, hidden_act="quick_gelu",
                                         layer_norm_eps=1e-5, attention_dropout=0.0)
    torch.manual_seed(0)
    hf = transformers.CLIPTextModel(hf_cfg).eval()
    ours = CLIPTextEncoder(OurClip(vocab_size=500, max_positions=77, dim=64, layers=2, heads=4, mlp=128,
                                   act="quick_gelu"), dtype=torch.float32).eval()
    missing = load_state(ours, hf.state_dict(), "clip", strict=False)
    assert not missing, missing
    ids = torch.randint(0, 500, (2, 77), generator=torch.Generator().manual_seed(2))
    with torch.no_grad():
        ref = hf(input_ids=ids, output_hidden_states=True)
        last, _ = ours(ids)
        pen, _ = ours(ids, output_hidden=-2)
    assert (last - ref.last_hidden_state).abs().max().item() < 1e-4
    # SDXL conditions on the penultimate layer's hidden state (before the final LayerNorm)
    assert (pen - ref.hidden_states[-2]).abs().max().item() < 1e-4


def test_openclip_bigg_matches_transformers_with_projection():
    """SDXL's second text tower (OpenCLIP bigG: exact-erf GELU, penultimate hidden state, pooled
    EOS row through ``text_projection``; ``models/text.py:90,119-143``) against
    ``transformers.CLIPTextModelWithProjection`` -- the conditioning of the reference's SDXL-base
    (``/root/reference/src/backend.py:24``).  The pooled ``text_embeds`` feed SDXL's add-embeds."""
    transformers = pytest.importorskip("transformers")
    from cassmantle_amd.models.text import CLIPTextConfig as OurClip
    V = 500
    hf_cfg = transformers.CLIPTextConfig(vocab_size=V, hidden_size=64, intermediate_size=160, num_hidden_layers=3,
                                         num_attention_heads=4, max_position_embeddings=77, hidden_act="gelu",
                                         layer_norm_eps=1e-5, attention_dropout=0.0, projection_dim=48,
                                         bos_token_id=V - 2, eos_token_id=V - 1, pad_token_id=V - 1)
    torch.manual_seed(0)
    hf = transformers.CLIPTextModelWithProjection(hf_cfg).eval()
    ours = CLIPTextEncoder(OurClip(vocab_size=V, max_positions=77, dim=64, layers=3, heads=4, mlp=160,
                                   act="gelu", projection_dim=48), dtype=torch.float32).eval()
    missing = load_state(ours, hf.state_dict(), "clip", strict=False)
    assert not missing, missing
    # real token layout: BOS, words, EOS, then EOS padding (SD pads with <|endoftext|>)
    texts = ["a gothic style piece depicting the following: a silent lantern tower", "river"]
    ids, _ = ours.tokenizer(texts, pad_to=77)
    assert ours.tokenizer.eos == V - 1 and (ids == V - 1).any(1).all()
    with torch.no_grad():
        ref = hf(input_ids=ids, output_hidden_states=True)
        pen, pooled = ours(ids, output_hidden=-2)
    assert (pen - ref.hidden_states[-2]).abs().max().item() < 1e-4
    assert pooled.shape == ref.text_embeds.shape
    assert (pooled - ref.text_embeds).abs().max().item() < 1e-4
    # the exporter is the inverse mapping for the projection too
    sd = export_diffusers(ours, "clip")
    assert torch.equal(sd["text_projection.weight"], hf.state_dict()["text_projection.weight"])

