"""Checkpoint I/O: map diffusers / transformers-format safetensors to the NHWC fused layout.

The framework runs random-init weights by default (BASELINE.json: no network, no checkpoints).
When real weights are available on disk (``ModelConfig.weights_path``), this module loads a
diffusers-style directory (``unet/``, ``vae/``, ``text_encoder/`` with ``*.safetensors``) or
individual files, converting on the fly:

* conv kernels ``[Cout, Cin, kh, kw]`` → ``[Cout, kh, kw, Cin]`` (K-contiguous implicit GEMM);
* 1×1 ``proj_in``/``proj_out`` convs → linear ``[Cout, Cin]``;
* separate ``to_q``/``to_k``/``to_v`` (or ``q_proj``/``k_proj``/``v_proj``) → one fused
  ``to_qkv`` (cross-attention: ``to_k``/``to_v`` → ``to_kv``);
* diffusers module paths → ours (``down_blocks.i`` → ``down.i``, ``mid_block.resnets.0`` →
  ``mid_res1``, ``time_embedding.linear_1`` → ``time_linear_1`` ...).

Only safetensors are read (no pickle).  :func:`export_diffusers` is the inverse mapping (used by
the tests to round-trip, and to hand weights back to other tools).
"""
from __future__ import annotations

import os
import re
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.nn as nn

# (regex on OUR name, replacement producing the diffusers name).  Applied in order.
_UNET_RULES: List[Tuple[str, str]] = [
    (r"^time_linear_(\d)\.", r"time_embedding.linear_\1."),
    (r"^add_linear_(\d)\.", r"add_embedding.linear_\1."),
    (r"^down\.(\d+)\.downsampler\.conv\.", r"down_blocks.\1.downsamplers.0.conv."),
    (r"^up\.(\d+)\.upsampler\.conv\.", r"up_blocks.\1.upsamplers.0.conv."),
    (r"^down\.(\d+)\.", r"down_blocks.\1."),
    (r"^up\.(\d+)\.", r"up_blocks.\1."),
    (r"^mid_res1\.", r"mid_block.resnets.0."),
    (r"^mid_res2\.", r"mid_block.resnets.1."),
    (r"^mid_attn\.", r"mid_block.attentions.0."),
    (r"\.ff\.proj_in\.", r".ff.net.0.proj."),
    (r"\.ff\.proj_out\.", r".ff.net.2."),
    (r"\.to_out\.", r".to_out.0."),
]
_VAE_RULES: List[Tuple[str, str]] = [
    (r"^post_quant_conv\.", r"post_quant_conv."),
    (r"^mid_res1\.", r"decoder.mid_block.resnets.0."),
    (r"^mid_res2\.", r"decoder.mid_block.resnets.1."),
    (r"^mid_attn\.", r"decoder.mid_block.attentions.0."),
    (r"^up\.(\d+)\.upsample_conv\.", r"decoder.up_blocks.\1.upsamplers.0.conv."),
    (r"^up\.(\d+)\.", r"decoder.up_blocks.\1."),
    (r"^(conv_in|conv_norm_out|conv_out)\.", r"decoder.\1."),
    (r"\.to_out\.", r".to_out.0."),
]
_CLIP_RULES: List[Tuple[str, str]] = [
    (r"^token_embedding$", r"text_model.embeddings.token_embedding.weight"),
    (r"^position_embedding$", r"text_model.embeddings.position_embedding.weight"),
    (r"^layers\.(\d+)\.self_attn\.to_out\.", r"text_model.encoder.layers.\1.self_attn.out_proj."),
    (r"^layers\.(\d+)\.", r"text_model.encoder.layers.\1.mlp." + "\x00"),
    (r"^final_layer_norm\.", r"text_model.final_layer_norm."),
    (r"^text_projection\.", r"text_projection."),
]


def _rename(name: str, rules: List[Tuple[str, str]]) -> str:
    for pat, rep in rules:
        new = re.sub(pat, rep, name)
        if new != name:
            name = new
    return name


def _clip_name(name: str) -> str:
    m = re.match(r"^layers\.(\d+)\.(.*)$", name)
    if m:
        i, rest = m.groups()
        base = f"text_model.encoder.layers.{i}."
        if rest.startswith("self_attn.to_out."):
            return base + "self_attn.out_proj." + rest.split(".")[-1]
        if rest.startswith("self_attn.to_qkv."):
            return base + "self_attn.qkv_proj." + rest.split(".")[-1]   # split on export
        if rest.startswith(("fc1.", "fc2.")):
            return base + "mlp." + rest
        return base + rest
    return _rename(name, [r for r in _CLIP_RULES if "\x00" not in r[1]])


def _is_conv(name: str, t: torch.Tensor) -> bool:
    return t.dim() == 4


def export_diffusers(model: nn.Module, kind: str) -> Dict[str, torch.Tensor]:
    """Our module -> diffusers/transformers-named state dict (NCHW convs, split QKV)."""
    out: Dict[str, torch.Tensor] = {}
    for name, t in model.state_dict().items():
        t = t.detach().cpu()
        if kind == "clip":
            dn = _clip_name(name)
        else:
            dn = _rename(name, _UNET_RULES if kind == "unet" else _VAE_RULES)
        if t.dim() == 4:
            t = t.permute(0, 3, 1, 2).contiguous()
        if ".attn2.to_kv." in dn:
            k, v = t.chunk(2, 0)
            out[dn.replace("to_kv", "to_k")] = k.contiguous()
            out[dn.replace("to_kv", "to_v")] = v.contiguous()
            continue
        if ".to_qkv." in dn or ".qkv_proj." in dn:
            q, k, v = t.chunk(3, 0)
            if ".qkv_proj." in dn:
                for nm, x in (("q_proj", q), ("k_proj", k), ("v_proj", v)):
                    out[dn.replace("qkv_proj", nm)] = x.contiguous()
            else:
                for nm, x in (("to_q", q), ("to_k", k), ("to_v", v)):
                    out[dn.replace("to_qkv", nm)] = x.contiguous()
            continue
        if kind == "unet" and re.search(r"\.(proj_in|proj_out)\.weight$", dn) and ".ff." not in dn and t.dim() == 2:
            t = t[:, :, None, None].contiguous()          # SD-1.5 stores 1x1 convs
        if kind == "vae" and dn.endswith("post_quant_conv.weight") and t.dim() == 2:
            t = t[:, :, None, None]
        out[dn] = t
    return out


def load_state(model: nn.Module, sd: Dict[str, torch.Tensor], kind: str, strict: bool = True) -> List[str]:
    """diffusers-named state dict -> our module (in place).  Returns missing names.  CLIP text
    towers are accepted with or without the ``text_model.`` prefix (checkpoint files carry it,
    a transformers>=5 ``CLIPTextModel.state_dict()`` does not)."""
    if kind == "clip" and not any(k.startswith("text_model.") for k in sd):
        sd = {("text_model." + k if k.startswith(("embeddings.", "encoder.", "final_layer_norm.")) else k): v
              for k, v in sd.items()}
    own = model.state_dict()
    missing = []
    with torch.no_grad():
        for name, dst in own.items():
            dn = _clip_name(name) if kind == "clip" else _rename(name, _UNET_RULES if kind == "unet" else _VAE_RULES)
            t: Optional[torch.Tensor] = None
            if ".attn2.to_kv." in dn:
                a, b = dn.replace("to_kv", "to_k"), dn.replace("to_kv", "to_v")
                if a in sd and b in sd:
                    t = torch.cat([sd[a], sd[b]], 0)
            elif ".to_qkv." in dn or ".qkv_proj." in dn:
                names = (["q_proj", "k_proj", "v_proj"] if ".qkv_proj." in dn else ["to_q", "to_k", "to_v"])
                key = "qkv_proj" if ".qkv_proj." in dn else "to_qkv"
                parts = [dn.replace(key, nm) for nm in names]
                if all(p in sd for p in parts):
                    t = torch.cat([sd[p] for p in parts], 0)
            elif dn in sd:
                t = sd[dn]
            if t is None:
                missing.append(dn)
                continue
            if t.dim() == 4 and dst.dim() == 4:
                t = t.permute(0, 2, 3, 1)
            elif t.dim() == 4 and dst.dim() == 2:
                t = t[:, :, 0, 0]
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"{name}: checkpoint {tuple(t.shape)} vs model {tuple(dst.shape)}")
            dst.copy_(t.to(dst.dtype))
    if strict and missing:
        raise KeyError(f"missing {len(missing)} tensors, e.g. {missing[:5]}")
    return missing


def load_causal_lm(model: nn.Module, sd: Dict[str, torch.Tensor]) -> List[str]:
    """HF Llama/Mistral layout (``model.layers.i.self_attn.q_proj.weight`` ...) ->
    :class:`~cassmantle_amd.models.lm.CausalLM`: q/k/v fused into ``qkv``, ``[up; gate]`` fused
    into ``gate_up`` (SwiGLU epilogue order).  Returns missing names."""
    missing: List[str] = []

    def get(name):
        t = sd.get(name)
        if t is None:
            missing.append(name)
        return t

    with torch.no_grad():
        def put(dst, t):
            if t is not None:
                if tuple(t.shape) != tuple(dst.shape):
                    raise ValueError(f"checkpoint {tuple(t.shape)} vs model {tuple(dst.shape)}")
                dst.copy_(t.to(dst.dtype))

        put(model.embed, get("model.embed_tokens.weight"))
        put(model.norm, get("model.norm.weight"))
        put(model.lm_head, sd.get("lm_head.weight", sd.get("model.embed_tokens.weight")))
        for i, blk in enumerate(model.blocks):
            p = f"model.layers.{i}."
            put(blk.attn_norm, get(p + "input_layernorm.weight"))
            put(blk.mlp_norm, get(p + "post_attention_layernorm.weight"))
            q, k, v = (get(p + f"self_attn.{n}_proj.weight") for n in ("q", "k", "v"))
            if q is not None and k is not None and v is not None:
                put(blk.qkv, torch.cat([q, k, v], 0))
            put(blk.o, get(p + "self_attn.o_proj.weight"))
            up, gate = get(p + "mlp.up_proj.weight"), get(p + "mlp.gate_proj.weight")
            if up is not None and gate is not None:
                put(blk.gate_up, torch.cat([up, gate], 0))
            put(blk.down, get(p + "mlp.down_proj.weight"))
    return missing


def export_causal_lm(model: nn.Module) -> Dict[str, torch.Tensor]:
    """Inverse of :func:`load_causal_lm` (HF names, split projections)."""
    c = model.c
    hd = c.head_dim
    out = {"model.embed_tokens.weight": model.embed, "model.norm.weight": model.norm,
           "lm_head.weight": model.lm_head}
    for i, blk in enumerate(model.blocks):
        p = f"model.layers.{i}."
        out[p + "input_layernorm.weight"] = blk.attn_norm
        out[p + "post_attention_layernorm.weight"] = blk.mlp_norm
        q, k, v = torch.split(blk.qkv, [c.heads * hd, c.kv_heads * hd, c.kv_heads * hd], 0)
        out[p + "self_attn.q_proj.weight"], out[p + "self_attn.k_proj.weight"] = q, k
        out[p + "self_attn.v_proj.weight"] = v
        out[p + "self_attn.o_proj.weight"] = blk.o
        up, gate = blk.gate_up.chunk(2, 0)
        out[p + "mlp.up_proj.weight"], out[p + "mlp.gate_proj.weight"] = up, gate
        out[p + "mlp.down_proj.weight"] = blk.down
    return {k: v.detach().cpu().contiguous() for k, v in out.items()}


# ---------------------------------------------------------------- BERT / MiniLM (guess scorer)
def _bert_pairs(model: nn.Module, prefix: str = "") -> List[Tuple[torch.Tensor, List[str]]]:
    """(our tensor, HF BertModel source names) — several sources are concatenated (fused QKV)."""
    p = prefix
    out = [(model.word_embeddings, [p + "embeddings.word_embeddings.weight"]),
           (model.position_embeddings, [p + "embeddings.position_embeddings.weight"]),
           (model.token_type_embeddings, [p + "embeddings.token_type_embeddings.weight"]),
           (model.emb_ln.weight, [p + "embeddings.LayerNorm.weight"]),
           (model.emb_ln.bias, [p + "embeddings.LayerNorm.bias"])]
    for i, blk in enumerate(model.layers):
        e = f"{p}encoder.layer.{i}."
        for kind in ("weight", "bias"):
            out.append((getattr(blk.attention.to_qkv, kind),
                        [e + f"attention.self.{n}.{kind}" for n in ("query", "key", "value")]))
            out.append((getattr(blk.attention.to_out, kind), [e + f"attention.output.dense.{kind}"]))
            out.append((getattr(blk.attention_ln, kind), [e + f"attention.output.LayerNorm.{kind}"]))
            out.append((getattr(blk.intermediate, kind), [e + f"intermediate.dense.{kind}"]))
            out.append((getattr(blk.output, kind), [e + f"output.dense.{kind}"]))
            out.append((getattr(blk.output_ln, kind), [e + f"output.LayerNorm.{kind}"]))
    return out


def load_bert(model: nn.Module, sd: Dict[str, torch.Tensor]) -> List[str]:
    """transformers ``BertModel`` / sentence-transformers MiniLM state dict -> our
    :class:`~cassmantle_amd.models.text.MiniLMEncoder` (query/key/value fused into ``to_qkv``).
    Accepts the bare, ``bert.`` and ``0.auto_model.`` key prefixes.  Returns missing names."""
    prefix = ""
    for cand in ("", "bert.", "0.auto_model.", "model."):
        if cand + "embeddings.word_embeddings.weight" in sd:
            prefix = cand
            break
    missing: List[str] = []
    with torch.no_grad():
        for dst, names in _bert_pairs(model, prefix):
            parts = [sd.get(n) for n in names]
            if any(t is None for t in parts):
                missing.extend(n for n, t in zip(names, parts) if t is None)
                continue
            t = parts[0] if len(parts) == 1 else torch.cat(parts, 0)
            if dst.shape[0] > t.shape[0] and dst.dim() == 2 and dst.shape[1] == t.shape[1] and "position" in names[0]:
                dst[: t.shape[0]].copy_(t.to(dst.dtype))       # shorter position table
                continue
            if tuple(t.shape) != tuple(dst.shape):
                raise ValueError(f"{names[0]}: checkpoint {tuple(t.shape)} vs model {tuple(dst.shape)}")
            dst.copy_(t.to(dst.dtype))
    return missing


def export_bert(model: nn.Module) -> Dict[str, torch.Tensor]:
    """Inverse of :func:`load_bert` (HF ``BertModel`` names, split Q/K/V)."""
    out: Dict[str, torch.Tensor] = {}
    for src, names in _bert_pairs(model):
        t = src.detach().cpu()
        for n, part in zip(names, t.chunk(len(names), 0)):
            out[n] = part.contiguous()
    return out


def read_safetensors(path: str) -> Dict[str, torch.Tensor]:
    from safetensors.torch import load_file
    if os.path.isdir(path):
        sd: Dict[str, torch.Tensor] = {}
        for fn in sorted(os.listdir(path)):
            if fn.endswith(".safetensors"):
                sd.update(load_file(os.path.join(path, fn)))
        return sd
    return load_file(path)


def load_pipeline_weights(sd_pipe, root: str) -> Dict[str, int]:
    """Load a diffusers-layout directory into a :class:`~cassmantle_amd.pipeline.StableDiffusion`.
    Returns the number of missing tensors per component found; raises if the directory holds
    none of ``unet/``, ``vae/``, ``text_encoder/`` (a wrong path must not silently keep random
    weights)."""
    if not any(os.path.exists(os.path.join(root, sub)) for sub in ("unet", "vae", "text_encoder")):
        raise FileNotFoundError(f"{root}: no unet/, vae/ or text_encoder/ safetensors directory")
    stats = {}
    for sub, model, kind in (("unet", sd_pipe.unet, "unet"), ("vae", sd_pipe.vae, "vae"),
                             ("text_encoder", sd_pipe.text_encoders[0], "clip")):
        p = os.path.join(root, sub)
        if os.path.exists(p):
            miss = load_state(model, read_safetensors(p), kind, strict=False)
            stats[sub] = len(miss)
    sd_pipe.unet.fuse_projections()   # refresh the fused time-embedding / context-K/V weights
    if hasattr(sd_pipe, "prepare"):
        sd_pipe.prepare()             # and the other derived weights (folds, parity convs, ...)
    if len(sd_pipe.text_encoders) > 1 and os.path.exists(os.path.join(root, "text_encoder_2")):
        miss = load_state(sd_pipe.text_encoders[1], read_safetensors(os.path.join(root, "text_encoder_2")), "clip",
                          strict=False)
        stats["text_encoder_2"] = len(miss)
    return stats
