"""A/B of the split-K UNet convs with and without fused GroupNorm output statistics (the
statistics ride the split-K reduce pass; prints us per call for each shape).

    python tools/ab_conv_stats.py
"""
import torch, sys, json
sys.path.insert(0, '.')
from cassmantle_amd import ops
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); e0=torch.cuda.Event(enable_timing=True); e1=torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it): fn()
    e1.record(); torch.cuda.synchronize(); return e0.elapsed_time(e1)/it*1e3
r=lambda *s, sc=1.0: (torch.randn(*s, device='cuda')*sc).to(torch.bfloat16)
for B,H,C in [(8,8,1280),(8,16,1280),(8,32,640)]:
    x=r(B,H,H,C); w=r(C,3,3,C,sc=(9*C)**-0.5); b=r(C,sc=0.1); st=ops.new_stats(B,C,'cuda')
    a=t(lambda: ops.conv2d(x,w,b)); s_=t(lambda: ops.conv2d(x,w,b,stats=st.zero_()))
    z=t(lambda: st.zero_())
    print(json.dumps({"conv":[B,H,C],"plain_us":round(a,1),"with_stats_us":round(s_-z,1)}))
