"""Per-row error of the bf16 attention forward vs a float64 reference (debug aid)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
import torch
from vspike import ops

def ref(qkv, B, N, H):
    D = H * 64
    x = qkv.double().view(B, N, 3, H, 64)
    q, k, v = (x[:, :, i].permute(0, 2, 1, 3) for i in range(3))
    s = (q @ k.transpose(-1, -2)) * 0.125
    return (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * N, D), torch.logsumexp(s, -1)

for (B, N, H) in [(1, 100, 1), (2, 196, 2), (1, 1568, 3), (2, 130, 1)]:
    g = torch.Generator().manual_seed(20)
    qkv = (torch.randn(B * N, 3 * H * 64, generator=g) * 1.5).to(torch.bfloat16)
    o = torch.empty(B * N, H * 64, dtype=torch.bfloat16, device="cuda")
    lse = torch.empty(B, H, N, device="cuda")
    ops.attn_fwd(qkv.cuda(), o, lse, B, N, H)
    o_ref, l_ref = ref(qkv, B, N, H)
    err = (o.double().cpu() - o_ref).norm(dim=1) / o_ref.norm(dim=1)
    lerr = (lse.double().cpu() - l_ref).abs().flatten()
    bad = torch.nonzero(err > 0.02).flatten().tolist()
    print(B, N, H, "rel", ((o.double().cpu() - o_ref).norm() / o_ref.norm()).item(), "bad rows", bad[:40], len(bad),
          "lse max err", lerr.max().item(), "at", lerr.argmax().item())
