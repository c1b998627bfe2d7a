import os, sys, torch
sys.path.insert(0, '.')
from cassmantle_amd.pipeline import SPECS, StableDiffusion
from cassmantle_amd.models.schedulers import make_plan
res = {}
sd_g = StableDiffusion(SPECS["tiny"], device="cuda", use_graphs=True, seed=5)
sd_e = StableDiffusion(SPECS["tiny"], device="cuda", use_graphs=False, seed=5)
plan = make_plan("pndm", 6, 7.5)
ctx, _ = sd_e.encode_prompt(["a castle"], "blurry")
x0 = sd_e.init_latents([7], plan)
a = sd_e.denoise(ctx, x0, plan).clone()
a2 = sd_e.denoise(ctx, x0, plan).clone()
b = sd_g.denoise(ctx, x0, plan).clone()
c = sd_g.denoise(ctx, x0, plan).clone()
print(os.environ.get("CASSMANTLE_LN_FOLD"), os.environ.get("CASSMANTLE_GN_FUSE"),
      "eager-eager", (a - a2).abs().max().item(), "eager-graph", (a - b).abs().max().item(),
      "graph-graph", (b - c).abs().max().item(), flush=True)
# single UNet eval eager vs same inputs
st = sd_e._states[list(sd_e._states)[0]]
