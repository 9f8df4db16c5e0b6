"""Linear plugin — drop-in for the reference's `src/model/linear.py:3-56` (NAME2MODEL['Linear']).

Same module tree and parameter names as the reference (`encoder.layers.{0,2,4}.weight/bias`,
`decoder.layers.{0,2,4}.*`, nn.ReLU at the odd indices), so a reference checkpoint's state_dict
loads unchanged.  The forward is ONE autograd node over the whole 6-layer MLP: every Linear runs
as an f32 MFMA GEMM with bias+ReLU fused in the epilogue, and the backward fuses each ReLU mask
into the dX GEMM that produces the masked gradient (VS_EPI_RELU_BWD).  The first layer's
K = frames*128*128 reduction (1,966,080 for the real `linear_video` config, a 503 M-parameter
weight) runs on the skinny split-K kernel (fragments streamed straight from HBM, fixed-order
partial sums, bias + ReLU in the reduce); its weight gradient (K = batch) is written with plain
stores.
"""
from __future__ import annotations

import math

import torch
from torch import nn

from . import _lib as L
from . import ops


class VsLinear(nn.Module):
    """nn.Linear-compatible parameter holder (weight [out, in], bias [out])."""

    def __init__(self, in_features: int, out_features: int):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features))
        self.bias = nn.Parameter(torch.empty(out_features))
        bound = 1.0 / math.sqrt(in_features)          # nn.Linear default init
        nn.init.uniform_(self.weight, -bound, bound)
        nn.init.uniform_(self.bias, -bound, bound)

    def extra_repr(self):
        return f"in_features={self.in_features}, out_features={self.out_features}"


def _mlp_stack(config) -> nn.Sequential:
    layer_num = config.layer_num if hasattr(config, "layer_num") else config["layer_num"]
    hidden = list(config["hidden_dims"])
    assert len(hidden) == layer_num, "hidden_dims must have the same length as layer_num"  # linear.py:22,43
    dims = [int(config["input_dim"])] + [int(h) for h in hidden] + [int(config["output_dim"])]
    seq = nn.Sequential()
    for i in range(len(dims) - 1):
        seq.append(VsLinear(dims[i], dims[i + 1]))
        if i < len(dims) - 2:
            seq.append(nn.ReLU())
    return seq


class Encoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.layers = _mlp_stack(config)


class Decoder(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.layers = _mlp_stack(config)


class Linear(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.encoder = Encoder(config["encoder"])
        self.decoder = Decoder(config["decoder"])
        self.output_dim = int(config["decoder"]["output_dim"]) // 100   # linear.py:8

    def _linears(self):
        lins, relu_after = [], []
        for stack in (self.encoder.layers, self.decoder.layers):
            mods = list(stack)
            for j, m in enumerate(mods):
                if isinstance(m, VsLinear):
                    lins.append(m)
                    relu_after.append(j + 1 < len(mods) and isinstance(mods[j + 1], nn.ReLU))
        return lins, relu_after

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        L.require_device(x)
        x = x.flatten(1).to(torch.float32).contiguous()                  # linear.py:11
        lins, relu = self._linears()
        params = []
        for m in lins:
            params += [m.weight, m.bias]
        y = _MLPFn.apply(x, tuple(relu), *params)
        return y.reshape(-1, 100, self.output_dim)                       # linear.py:14


class _MLPFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, relu, *params):
        ws, bs = params[0::2], params[1::2]
        outs = []
        h = x
        for w, b, r in zip(ws, bs, relu):
            M, K = h.shape
            N = w.shape[0]
            # the skinny split-K path of vs_gemm (gemm_dw.hip skinny_ok): M <= 16 and N <= 256 (or
            # M, N <= 64), K % 16 == 0
            skinny = K >= 16384 and K % 16 == 0 and N % 16 == 0 and ((M <= 16 and N <= 256) or (M <= 64 and N <= 64))
            nb = ops.splitk_workspace_bytes(torch.float32, M, N, K) if skinny else 0
            if nb:
                # long reduction (the first layer: K = frames*H*W, 1,966,080 for linear_video): skinny
                # split-K streaming the weight at the HBM rate, splits summed in a fixed order; bias
                # (and ReLU) applied by the split reduce
                y = torch.zeros(M, N, dtype=torch.float32, device=h.device)
                wsp = torch.empty(nb // 4 + 4, dtype=torch.float32, device=h.device)
                ops.gemm(h, w.detach(), y, M=M, N=N, K=K, a_kcontig=True, b_kcontig=True, lda=h.stride(0),
                         ldb=w.stride(0), ldc=N, epilogue=L.EPI_ATOMIC | L.EPI_BIAS | (L.EPI_RELU if r else 0),
                         bias=b.detach(), workspace=wsp)
            else:
                y = torch.empty(M, N, dtype=torch.float32, device=h.device)
                ops.linear(h, w.detach(), y, bias=b.detach(), epilogue=L.EPI_RELU if r else 0)
            outs.append(y)
            h = y
        ctx.save_for_backward(x, *outs, *[w.detach() for w in ws])
        ctx.relu = relu
        ctx.n = len(ws)
        ctx.need_x = ctx.needs_input_grad[0]
        return h

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g):
        n = ctx.n
        saved = ctx.saved_tensors
        x, outs, ws = saved[0], saved[1:1 + n], saved[1 + n:]
        relu = ctx.relu
        grads = [None] * (2 * n)
        dy = g.contiguous().to(torch.float32)
        for i in reversed(range(n)):
            inp = x if i == 0 else outs[i - 1]
            # K = batch: one split, plain stores (f32 atomics on the 503 M-element first-layer
            # gradient would run at ~1.3 TB/s instead of the store rate); db fused as row sums
            dw = torch.empty_like(ws[i])
            db = torch.zeros(ws[i].shape[0], dtype=torch.float32, device=dy.device)
            ops.linear_dw(dy, inp, dw, db=db, accumulate=False)
            grads[2 * i], grads[2 * i + 1] = dw, db
            if i > 0 or ctx.need_x:
                dx = torch.empty(dy.shape[0], ws[i].shape[1], dtype=torch.float32, device=dy.device)
                if i > 0 and relu[i - 1]:
                    # the gradient flows through the previous layer's ReLU: mask fused here
                    ops.linear_dx(dy, ws[i], dx, epilogue=L.EPI_RELU_BWD, aux_in=outs[i - 1],
                                  ld_aux_in=outs[i - 1].stride(0))
                else:
                    ops.linear_dx(dy, ws[i], dx)
                dy = dx
        dx_in = dy if ctx.need_x else None
        return (dx_in, None, *grads)
