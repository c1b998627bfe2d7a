"""Localise a stage-overlap mismatch: serial vs serial (second instance) vs overlapped, per
generation, latents (UNet output) and images (VAE output) compared separately."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cassmantle_amd.pipeline import SPECS, StableDiffusion  # noqa: E402

prompts = [["a lantern", "a river"], ["an ember", "a tower"], ["a shadow", "a forest"]]


def run(sd, sync):
    lat, img = [], []
    for i, p in enumerate(prompts):
        im = sd.generate_tensor(p, "blurry", [i, i + 10], steps=6, sync_caller=sync)
        lat.append(sd.last_latents)
        img.append(im)
        if sync:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return [l.clone() for l in lat], [x.clone() for x in img]


def cmp(tag, A, B):
    (la, ia), (lb, ib) = A, B
    for i in range(len(la)):
        dl = (la[i].float() - lb[i].float()).abs()
        di = (ia[i].float() - ib[i].float()).abs()
        print(f"{tag} gen{i}: latents equal={torch.equal(la[i], lb[i])} max={dl.max().item():.3g} "
              f"nz={int((dl > 0).sum())}/{dl.numel()} | image equal={torch.equal(ia[i], ib[i])} "
              f"max={di.max().item():.0f} nz={int((di > 0).sum())}", flush=True)


knobs = {k: v for k, v in os.environ.items() if k.startswith("CASSMANTLE_")}
print("knobs", knobs, flush=True)
b = StableDiffusion(SPECS["sd15"], device="cuda", seed=0, overlap_decode=False)
R1 = run(b, True)
R1b = run(b, True)
cmp("serial-vs-serial(same inst)", R1, R1b)
b2 = StableDiffusion(SPECS["sd15"], device="cuda", seed=0, overlap_decode=False)
cmp("serial-vs-serial(new inst)", R1, run(b2, True))
a = StableDiffusion(SPECS["sd15"], device="cuda", seed=0, overlap_decode=True)
cmp("overlap(sync)-vs-serial", R1, run(a, True))
cmp("overlap(async)-vs-serial", R1, run(a, False))
cmp("serial(async)-vs-serial", R1, run(b, False))
