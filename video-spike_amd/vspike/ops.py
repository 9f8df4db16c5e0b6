"""Tensor-level wrappers over the libvspike C-ABI (one function per entry point).

Each wrapper validates devices, passes raw pointers + sizes and enqueues on the current stream.
Outputs are caller-allocated tensors (the PyTorch caching allocator owns all memory).
"""
from __future__ import annotations

import ctypes
import math

import torch

from . import _lib as L
from ._lib import check, lib, ptr, require_device, stream


def gemm(a, b, c, *, M, N, K, a_kcontig, b_kcontig, lda, ldb, ldc, epilogue=0, alpha=1.0, bias=None,
         residual=None, ld_residual=0, pos=None, pos_rows=0, aux_in=None, ld_aux_in=0, aux_out=None,
         ld_aux_out=0, split_k=0, a_rowsum=None, workspace=None):
    """C[M,N] = epilogue(alpha * A @ B); layouts as in include/vspike.h (vs_gemm).
    workspace: optional device tensor for split-K partials of an ATOMIC GEMM (see vs_gemm_desc)."""
    require_device(a, b, c)
    d = L.GemmDesc()
    d.dtype = L.dtype_code(a.dtype)
    if L.dtype_code(b.dtype) != d.dtype:
        raise L.VsError("gemm: A and B must share a dtype")
    d.out_dtype = L.dtype_code(c.dtype)
    d.a_kcontig, d.b_kcontig = int(a_kcontig), int(b_kcontig)
    d.M, d.N, d.K = M, N, K
    d.a, d.lda, d.b, d.ldb, d.c, d.ldc = a.data_ptr(), lda, b.data_ptr(), ldb, c.data_ptr(), ldc
    d.epilogue, d.alpha = epilogue, alpha
    d.bias = ptr(bias)
    d.residual, d.ld_residual = ptr(residual), ld_residual
    d.pos, d.pos_rows = ptr(pos), pos_rows
    d.aux_in, d.ld_aux_in = ptr(aux_in), ld_aux_in
    d.aux_out, d.ld_aux_out = ptr(aux_out), ld_aux_out
    d.split_k = split_k
    d.a_rowsum = ptr(a_rowsum)
    if workspace is not None:
        d.workspace, d.workspace_bytes = workspace.data_ptr(), workspace.numel() * workspace.element_size()
    check(lib().vs_gemm(ctypes.byref(d), stream()), "vs_gemm")
    return c


def linear(x, w, out, *, bias=None, epilogue=0, **kw):
    """out[M,N] = x[M,K] @ w[N,K]^T (+ epilogue): the nn.Linear forward."""
    M, K = x.shape
    N = w.shape[0]
    if bias is not None:
        epilogue |= L.EPI_BIAS
    return gemm(x, w, out, M=M, N=N, K=K, a_kcontig=True, b_kcontig=True, lda=x.stride(0), ldb=w.stride(0),
                ldc=out.stride(0), epilogue=epilogue, bias=bias, **kw)


def quant_mxfp8(x, q, scales):
    """MX-FP8 quantisation (vs_quant_mxfp8): x [M, K] f32/bf16 -> q [M, K] uint8 (OCP e4m3 codes) and
    scales [M, K // 32] uint8 (E8M0 exponents, 2^(e - 127) per 32 consecutive elements of a row)."""
    require_device(x, q, scales)
    M, K = x.shape
    check(lib().vs_quant_mxfp8(L.dtype_code(x.dtype), M, K, x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0),
                               scales.data_ptr(), scales.stride(0), stream()), "vs_quant_mxfp8")
    return q, scales


def gemm_mxfp8(a_q, a_s, b_q, b_s, c, *, epilogue=0, bias=None, residual=None, aux_out=None, alpha=1.0):
    """c = epilogue(A B^T) on the block-scaled fp8 MFMA (vs_gemm_mxfp8): a_q [M, K], b_q [N, K] uint8
    e4m3 codes with their E8M0 scales (quant_mxfp8 layout); c [M, N] f32 or bf16."""
    require_device(a_q, b_q, c)
    M, K = a_q.shape
    N = b_q.shape[0]
    d = L.GemmDesc()
    d.dtype, d.out_dtype = L.VS_FP8, L.dtype_code(c.dtype)
    d.a_kcontig = d.b_kcontig = 1
    d.M, d.N, d.K = M, N, K
    d.a, d.lda, d.b, d.ldb, d.c, d.ldc = a_q.data_ptr(), a_q.stride(0), b_q.data_ptr(), b_q.stride(0), c.data_ptr(), c.stride(0)
    d.epilogue, d.alpha = epilogue, alpha
    d.bias = ptr(bias)
    d.residual, d.ld_residual = ptr(residual), (residual.stride(0) if residual is not None else 0)
    d.aux_out, d.ld_aux_out = ptr(aux_out), (aux_out.stride(0) if aux_out is not None else 0)
    check(lib().vs_gemm_mxfp8(ctypes.byref(d), a_s.data_ptr(), a_s.stride(0), b_s.data_ptr(), b_s.stride(0), stream()),
          "vs_gemm_mxfp8")
    return c


def mlp_fused_ok(M: int, D: int, F: int) -> bool:
    """vs_mlp_fused_ok: the fused MLP kernels take this shape (bf16, D = 192, F % 64 == 0)."""
    return bool(lib().vs_mlp_fused_ok(int(M), int(D), int(F)))


def mlp_fwd(h2, w1, b1, w2, b2, y, out):
    """out = y + gelu(h2 @ w1^T + b1) @ w2^T + b2 in one launch (vs_mlp_fwd): h2 [M, D] bf16, w1 [F, D],
    w2 [D, F] bf16, y / out [M, D] f32 (modeling_videomae.py:370-399)."""
    require_device(h2, w1, w2, y, out)
    M, D = h2.shape
    F = w1.shape[0]
    check(lib().vs_mlp_fwd(M, D, F, h2.data_ptr(), h2.stride(0), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                           b2.data_ptr(), y.data_ptr(), y.stride(0), out.data_ptr(), out.stride(0), stream()),
          "vs_mlp_fwd")
    return out


def mlp_bwd_da(h2, w1, b1, w2, dy, da, a):
    """da = (dy @ w2) * gelu'(h2 @ w1^T + b1) and a = gelu(h2 @ w1^T + b1), the pre-activation
    recomputed (vs_mlp_bwd_da): dy [M, D] bf16, da / a [M, F] bf16."""
    require_device(h2, w1, w2, dy, da, a)
    M, D = h2.shape
    F = w1.shape[0]
    check(lib().vs_mlp_bwd_da(M, D, F, h2.data_ptr(), h2.stride(0), w1.data_ptr(), b1.data_ptr(), w2.data_ptr(),
                              dy.data_ptr(), dy.stride(0), da.data_ptr(), da.stride(0), a.data_ptr(), a.stride(0),
                              stream()), "vs_mlp_bwd_da")
    return da, a


def linear_dx(dy, w, out, *, epilogue=0, accumulate=False, **kw):
    """out[M,K] = dy[M,N] @ w[N,K]; accumulate=True adds into an f32 `out` with split-K atomics
    (for skinny products whose reduction N is long, e.g. the head's dZ over 100*neurons)."""
    M, N = dy.shape
    K = w.shape[1]
    if accumulate:
        epilogue |= L.EPI_ATOMIC
    return gemm(dy, w, out, M=M, N=K, K=N, a_kcontig=True, b_kcontig=False, lda=dy.stride(0), ldb=w.stride(0),
                ldc=out.stride(0), epilogue=epilogue, **kw)


def splitk_workspace_bytes(dtype, M, N, K):
    return int(lib().vs_gemm_splitk_workspace_bytes(L.dtype_code(dtype), M, N, K))


def linear_dw(dy, x, dw, *, accumulate=True, db=None, workspace=None):
    """dw[N,K] (+)= dy[M,N]^T @ x[M,K]  (f32 dw, split-K over the M reduction).
    db (optional, f32 [N]) += column sums of dy, fused into the same pass.  The splits are summed
    through `workspace` (allocated here when None; False = f32 atomics instead)."""
    M, N = dy.shape
    K = x.shape[1]
    epi = L.EPI_ATOMIC if accumulate else 0
    if accumulate and workspace is None:
        nb = splitk_workspace_bytes(dy.dtype, N, K, M)
        workspace = torch.empty(nb // 4 + 4, dtype=torch.float32, device=dy.device) if nb else None
    ws = None if workspace is False else workspace
    return gemm(dy, x, dw, M=N, N=K, K=M, a_kcontig=False, b_kcontig=False, lda=dy.stride(0), ldb=x.stride(0),
                ldc=dw.stride(0), epilogue=epi, split_k=0 if accumulate else 1, a_rowsum=db, workspace=ws)


def layernorm_fwd(x, gamma, beta, eps, y, mean, rstd):
    require_device(x, y)
    rows, cols = x.shape
    check(lib().vs_layernorm_fwd(L.dtype_code(y.dtype), rows, cols, x.data_ptr(), x.stride(0), gamma.data_ptr(),
                                 beta.data_ptr(), eps, y.data_ptr(), y.stride(0), mean.data_ptr(), rstd.data_ptr(),
                                 stream()), "vs_layernorm_fwd")
    return y


def layernorm_bwd_workspace_bytes(rows, cols):
    return int(lib().vs_layernorm_bwd_workspace_bytes(rows, cols))


def layernorm_bwd(dy, x, mean, rstd, gamma, dx, dgamma, dbeta, dres=None, dx_lp=None, workspace=None):
    """LayerNorm backward (dy f32 or bf16); dgamma/dbeta accumulate.  `workspace` (f32, >= layernorm_bwd_workspace_bytes)
    is allocated here when not given; pass False to use the per-block atomic reduction instead."""
    require_device(dy, x, dx)
    rows, cols = x.shape
    if workspace is None:
        workspace = torch.empty(layernorm_bwd_workspace_bytes(rows, cols) // 4 + 4, dtype=torch.float32,
                                device=x.device)
    ws = None if workspace is False else workspace
    check(lib().vs_layernorm_bwd_dt(L.dtype_code(dy.dtype), rows, cols, dy.data_ptr(), dy.stride(0), x.data_ptr(),
                                    x.stride(0), mean.data_ptr(), rstd.data_ptr(), gamma.data_ptr(), ptr(dres),
                                    dres.stride(0) if dres is not None else 0, dx.data_ptr(), dx.stride(0), ptr(dx_lp),
                                    dgamma.data_ptr(), dbeta.data_ptr(), ptr(ws), stream()), "vs_layernorm_bwd")
    return dx


def linear_dx_ln_bwd(dy, w, x, mean, rstd, gamma, dx, dgamma, dbeta, *, dres=None, dx_lp=None, scratch=None,
                     workspace=None):
    """dx = dres + LN'(dy @ w; x, mean, rstd, gamma), dgamma/dbeta accumulate (vs_gemm_ln_bwd): the
    dX product of a Linear fused with the backward of the LayerNorm that feeds it.  dy [M, Nout]
    (bf16 or f32), w [Nout, D]; `scratch` ([M, D] f32) is only written off the fused path."""
    require_device(dy, w, x, dx)
    M, Nout = dy.shape
    D = w.shape[1]
    if scratch is None:
        scratch = torch.empty(M, D, dtype=torch.float32, device=x.device)
    if workspace is None:
        workspace = torch.empty(layernorm_bwd_workspace_bytes(M, D) // 4 + 4, dtype=torch.float32, device=x.device)
    d = L.GemmDesc()
    d.dtype = L.dtype_code(dy.dtype)
    d.out_dtype = L.dtype_code(torch.float32)
    d.a_kcontig, d.b_kcontig = 1, 0
    d.M, d.N, d.K = M, D, Nout
    d.a, d.lda, d.b, d.ldb, d.c, d.ldc = dy.data_ptr(), dy.stride(0), w.data_ptr(), w.stride(0), scratch.data_ptr(), D
    d.alpha = 1.0
    check(lib().vs_gemm_ln_bwd(ctypes.byref(d), x.data_ptr(), x.stride(0), mean.data_ptr(), rstd.data_ptr(),
                               gamma.data_ptr(), ptr(dres), dres.stride(0) if dres is not None else 0, dx.data_ptr(),
                               dx.stride(0), ptr(dx_lp), dgamma.data_ptr(), dbeta.data_ptr(), workspace.data_ptr(),
                               stream()), "vs_gemm_ln_bwd")
    return dx


def linear_ln_fwd(x, w, y, residual, gamma, beta, eps, h, mean, rstd, *, bias=None):
    """y = x @ w^T (+ bias) + residual (f32) and h = LayerNorm(y) (bf16) with its row mean / rstd
    (vs_gemm_ln_fwd): the ViT block's attention-output product fused with layernorm_after."""
    require_device(x, w, y, residual, h)
    M, K = x.shape
    N = w.shape[0]
    d = L.GemmDesc()
    d.dtype = L.dtype_code(x.dtype)
    d.out_dtype = L.dtype_code(torch.float32)
    d.a_kcontig, d.b_kcontig = 1, 1
    d.M, d.N, d.K = M, N, K
    d.a, d.lda, d.b, d.ldb, d.c, d.ldc = x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), y.data_ptr(), y.stride(0)
    d.alpha = 1.0
    d.epilogue = L.EPI_RESIDUAL | (L.EPI_BIAS if bias is not None else 0)
    d.bias = ptr(bias)
    d.residual, d.ld_residual = residual.data_ptr(), residual.stride(0)
    check(lib().vs_gemm_ln_fwd(ctypes.byref(d), gamma.data_ptr(), beta.data_ptr(), float(eps), h.data_ptr(),
                               h.stride(0), mean.data_ptr(), rstd.data_ptr(), stream()), "vs_gemm_ln_fwd")
    return h


def attn_fwd(qkv, o, lse, B, N, H, scale=0.125):
    require_device(qkv, o, lse)
    check(lib().vs_attn_fwd(L.dtype_code(qkv.dtype), B, N, H, 64, qkv.data_ptr(), qkv.stride(0), o.data_ptr(),
                            o.stride(0), lse.data_ptr(), scale, stream()), "vs_attn_fwd")
    return o


def attn_bwd_workspace_bytes(B, N, H):
    return int(lib().vs_attn_bwd_workspace_bytes(B, N, H, 64))


def attn_bwd(qkv, o, dout, lse, dqkv, workspace, B, N, H, scale=0.125):
    require_device(qkv, o, dout, lse, dqkv, workspace)
    check(lib().vs_attn_bwd(L.dtype_code(qkv.dtype), B, N, H, 64, qkv.data_ptr(), qkv.stride(0), o.data_ptr(),
                            o.stride(0), dout.data_ptr(), dout.stride(0), lse.data_ptr(), dqkv.data_ptr(),
                            dqkv.stride(0), workspace.data_ptr(), scale, stream()), "vs_attn_bwd")
    return dqkv


def patch_im2col(pixels, cols, tubelet, patch):
    require_device(pixels, cols)
    B, F, C, H, W = pixels.shape
    check(lib().vs_patch_im2col(L.dtype_code(cols.dtype), B, F, C, H, W, tubelet, patch, pixels.data_ptr(),
                                cols.data_ptr(), stream()), "vs_patch_im2col")
    return cols


def patch_embed_fwd(pixels, weight, bias, pos, out, tubelet, patch, cols=None):
    """out[B*n_tok, D] f32 = Conv3d patch embedding of pixels (B, F, C, H, W) f32 + bias + pos, with the
    tubelet gather inside the GEMM (vs_patch_embed_fwd); cols (optional bf16 [B*n_tok, C*t*p*p])
    receives the gathered rows for the weight gradient."""
    require_device(pixels, weight, bias, pos, out)
    B, F, C, H, W = pixels.shape
    check(lib().vs_patch_embed_fwd(B, F, C, H, W, tubelet, patch, pixels.data_ptr(), weight.data_ptr(), bias.data_ptr(),
                                   pos.data_ptr(), out.shape[1], out.data_ptr(), ptr(cols), stream()),
          "vs_patch_embed_fwd")
    return out


def patch_embed_fused_ok(cfg, dtype) -> bool:
    """Shapes the fused patch embedding covers (else im2col + GEMM)."""
    return (dtype == torch.bfloat16 and cfg.tubelet_size == 2 and cfg.patch_size == 16 and
            cfg.hidden_size in (64, 128, 192) and cfg.num_channels <= 8 and L.knob_get("no_patch_fused") == 0)


def patch_embed_dw_workspace_bytes(tokens, D, K):
    return int(lib().vs_patch_embed_dw_workspace_bytes(tokens, D, K))


def patch_dw_ok(cfg, dtype) -> bool:
    """Shapes the gather weight gradient covers (else im2col + the dW product of vs_gemm)."""
    return (dtype == torch.bfloat16 and cfg.tubelet_size == 2 and cfg.patch_size == 16 and cfg.hidden_size % 64 == 0
            and cfg.num_channels <= 8 and cfg.hidden_size <= cfg.num_channels * 512
            and L.knob_get("no_patch_fused") == 0)


def patch_embed_dw(pixels, dx, dweight, dbias, tubelet, patch, workspace=None):
    """dweight[D, C*t*p*p] += dx^T X and dbias[D] += column sums of dx, X the tubelet gather of the f32
    pixels (B, F, C, H, W) read in the operand load (vs_patch_embed_dw); dx bf16 [B*n_tok, D]."""
    require_device(pixels, dx, dweight)
    B, F, C, H, W = pixels.shape
    D = dx.shape[1]
    K = dweight.shape[1]
    if workspace is None:
        workspace = torch.empty(patch_embed_dw_workspace_bytes(dx.shape[0], D, K) // 4 + 4, dtype=torch.float32,
                                device=dx.device)
    check(lib().vs_patch_embed_dw(B, F, C, H, W, tubelet, patch, pixels.data_ptr(), dx.data_ptr(), dx.stride(0), D,
                                  dweight.data_ptr(), dweight.stride(0), ptr(dbias), workspace.data_ptr(),
                                  workspace.numel() * 4, stream()), "vs_patch_embed_dw")
    return dweight


def sinusoid_table(n_pos, dim, device):
    out = torch.empty(n_pos, dim, dtype=torch.float32, device=device)
    check(lib().vs_sinusoid_table(n_pos, dim, out.data_ptr(), stream()), "vs_sinusoid_table")
    return out


def colsum(x, out, rows=None, cols=None):
    """out[c] += sum_r x[r, c] (out f32)."""
    require_device(x, out)
    rows = x.shape[0] if rows is None else rows
    cols = x.shape[1] if cols is None else cols
    check(lib().vs_colsum(L.dtype_code(x.dtype), rows, cols, x.data_ptr(), x.stride(0), out.data_ptr(), stream()),
          "vs_colsum")
    return out


def cast(x, out):
    require_device(x, out)
    check(lib().vs_cast(L.dtype_code(x.dtype), L.dtype_code(out.dtype), x.numel(), x.data_ptr(), out.data_ptr(),
                        stream()), "vs_cast")
    return out


def poisson_nll(log_rate, target, loss_out, dx=None, grad_scale=1.0, workspace=None):
    require_device(log_rate, target, loss_out)
    n = log_rate.numel()
    if workspace is None:
        workspace = torch.empty(int(lib().vs_poisson_workspace_bytes(n)) // 4, dtype=torch.float32,
                                device=log_rate.device)
    check(lib().vs_poisson_nll(n, log_rate.data_ptr(), target.data_ptr(), loss_out.data_ptr(), ptr(dx), grad_scale,
                               workspace.data_ptr(), stream()), "vs_poisson_nll")
    return loss_out


def poisson_nll_bwd(log_rate, target, grad_out, dx):
    require_device(log_rate, target, grad_out, dx)
    check(lib().vs_poisson_nll_bwd(log_rate.numel(), log_rate.data_ptr(), target.data_ptr(), grad_out.data_ptr(),
                                   dx.data_ptr(), stream()), "vs_poisson_nll_bwd")
    return dx


def mse_loss(pred, target, loss_out, dx=None, grad_scale=1.0, workspace=None):
    """mean((pred - target)^2) into loss_out (device scalar); dx = grad_scale * 2 (pred - target) / n."""
    require_device(pred, target, loss_out)
    n = pred.numel()
    if workspace is None:
        workspace = torch.empty(int(lib().vs_poisson_workspace_bytes(n)) // 4, dtype=torch.float32, device=pred.device)
    check(lib().vs_mse_loss(n, pred.data_ptr(), target.data_ptr(), loss_out.data_ptr(), ptr(dx), grad_scale,
                            workspace.data_ptr(), stream()), "vs_mse_loss")
    return loss_out


def mse_loss_bwd(pred, target, grad_out, dx):
    require_device(pred, target, grad_out, dx)
    check(lib().vs_mse_loss_bwd(pred.numel(), pred.data_ptr(), target.data_ptr(), grad_out.data_ptr(), dx.data_ptr(),
                                stream()), "vs_mse_loss_bwd")
    return dx


def adamw(param, grad, exp_avg, exp_avg_sq, hyper, param_lp=None):
    require_device(param, grad, exp_avg, exp_avg_sq, hyper)
    check(lib().vs_adamw(param.numel(), param.data_ptr(), grad.data_ptr(), exp_avg.data_ptr(), exp_avg_sq.data_ptr(),
                         ptr(param_lp), hyper.data_ptr(), stream()), "vs_adamw")


def vit_layer_fwd(layer_struct):
    check(lib().vs_vit_layer_fwd(ctypes.byref(layer_struct), stream()), "vs_vit_layer_fwd")


def vit_layer_bwd(layer_struct, grad_struct):
    check(lib().vs_vit_layer_bwd(ctypes.byref(layer_struct), ctypes.byref(grad_struct), stream()),
          "vs_vit_layer_bwd")


# ---- timing (bench instrumentation) -----------------------------------------------------------
def timing_enable(mask: int):
    """mask: OR of (1 << TIMER_*); 0 disables and discards recorded events."""
    check(lib().vs_timing_enable(int(mask)), "vs_timing_enable")


def timing_collect(timer: int, with_bytes: bool = False):
    """(launches, total ms) of one timer, and its total algorithmic bytes with `with_bytes`."""
    n = ctypes.c_int64(0)
    ms = ctypes.c_double(0.0)
    nb = ctypes.c_double(0.0)
    check(lib().vs_timing_bytes(timer, ctypes.byref(nb)), "vs_timing_bytes")
    check(lib().vs_timing_collect(timer, ctypes.byref(n), ctypes.byref(ms)), "vs_timing_collect")
    return (int(n.value), float(ms.value), float(nb.value)) if with_bytes else (int(n.value), float(ms.value))


def attn_scale(head_dim: int = 64) -> float:
    return 1.0 / math.sqrt(head_dim)


def video_preprocess(video, frame_idx, size=224, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225), out=None):
    """K0 on the device (videomae.py:18-25): raw (B, T, 1, H, W) float32 (integer-valued 0..255) or
    uint8 video -> pixel_values (B, len(frame_idx), 3, size, size) f32, bit-identical to the
    reference's HF image processor.  frame_idx: host sequence of source frame indices."""
    require_device(video)
    if video.dim() != 5 or video.shape[2] != 1:
        raise L.VsError("video_preprocess: expected (B, T, 1, H, W)")
    if video.dtype == torch.uint8:
        code = L.VS_U8
    elif video.dtype == torch.float32:
        code = L.VS_F32
    else:
        raise L.VsError("video_preprocess: float32 or uint8 frames")
    video = video.contiguous()
    B, T, _, H, W = video.shape
    idx = [int(i) for i in frame_idx]
    if out is None:
        out = torch.empty(B, len(idx), 3, size, size, dtype=torch.float32, device=video.device)
    fi = (ctypes.c_int32 * len(idx))(*idx)
    m = (ctypes.c_float * 3)(*[float(v) for v in mean])
    sd = (ctypes.c_float * 3)(*[float(v) for v in std])
    check(lib().vs_video_preprocess(code, B, T, H, W, video.data_ptr(), fi, len(idx), size, m, sd, out.data_ptr(),
                                    stream()), "vs_video_preprocess")
    return out
