"""Q = 0, V = 1: every p = 1, so O = N / l_kernel exposes the kernel's row sums (debug aid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
import torch
from vspike import ops
for N in (64, 128):
    qkv = torch.zeros(N, 192)
    qkv[:, 64:128] = torch.randn(N, 64)
    qkv[:, 128:] = 1.0
    qkv = qkv.to(torch.bfloat16).cuda()
    o = torch.empty(N, 64, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(1, 1, N, device="cuda")
    ops.attn_fwd(qkv, o, lse, 1, N, 1)
    print(N, "l = N/O per query:", [round(N / float(x), 2) for x in o[:, 0].cpu()[:40]])
    print(N, "exp(lse):", [round(float(x), 2) for x in lse.exp().flatten().cpu()[:40]])
