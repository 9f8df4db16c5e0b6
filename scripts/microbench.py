"""Per-op timing of the ViT training-step shapes (C2: ViT-Tiny, B=16) with hipEvents.

Prints, per op: average microseconds over `--reps` launches, algorithmic HBM bytes and FLOPs,
achieved GB/s and TFLOP/s, and the fraction of the op's bound (HBM 6.3 TB/s measured-achievable
or 2.5 PF bf16 MFMA).  Usage:  python scripts/microbench.py [--only gemm|attn|ln] [--reps 50]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from vspike import _lib as L, ops  # noqa: E402

HBM = 6.3e12
MFMA = 2.5e15


COLD = None


def timeit(fn, reps):
    if fn is None:
        return float("nan")
    for _ in range(3):
        fn()
    if COLD is not None:  # every rep from cold caches: a 512-MB fill evicts L2 and the Infinity Cache first
        tot = 0.0
        for _ in range(reps):
            COLD.fill_(1.0)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            tot += s.elapsed_time(e)
        return tot / reps * 1e3
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


SELECT = ""


def report(name, us, nbytes, flops):
    gbs = nbytes / (us * 1e-6) / 1e9
    tfs = flops / (us * 1e-6) / 1e12
    bound = max(nbytes / HBM, flops / MFMA) * 1e6
    print(f"{name:34s} {us:9.1f} us  {gbs:8.0f} GB/s  {tfs:7.1f} TF/s  bound {bound:7.1f} us  ({bound / us * 100:5.1f}% of roof)")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="", help="gemm|attn|ln, or gemm:<name substring> for one GEMM")
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--heads", type=int, default=3, help="attention heads (3: C2 ViT-Tiny, 12: C3 ViT-Base)")
    ap.add_argument("--attn-variants", default="0",
                    help="VS_KNOB_ATTN_VARIANT values, comma-separated (low nibble: forward kernel, bits 4-7: backward)")
    ap.add_argument("--attn-scale", type=float, default=3.0, help="q, k, v ~ N(0, scale^2)")
    ap.add_argument("--cold", action="store_true", help="evict L2 / Infinity Cache before every timed launch")
    ap.add_argument("--ln-dim", type=int, default=192, help="LayerNorm width of --only ln (768: C3 / C5)")
    a = ap.parse_args()
    global COLD
    if a.cold:
        COLD = torch.empty(128 * 1024 * 1024, device="cuda")
    global SELECT
    if a.only.startswith("gemm:"):
        a.only, SELECT = "gemm", a.only[5:]
    dev = "cuda"
    B, N, D, F, H = a.batch, 1568, 192, 768, a.heads
    M = B * N
    bf = torch.bfloat16
    r = lambda *s, dt=bf: (torch.randn(*s, device=dev) * 0.5).to(dt)  # noqa: E731
    if a.only in ("", "gemm"):
        x, w3, wd, w1, w2 = r(M, D), r(3 * D, D), r(D, D), r(F, D), r(D, F)
        b3, bd, b1 = r(3 * D, dt=torch.float32), r(D, dt=torch.float32), r(F, dt=torch.float32)
        qkv, o, a_, pre = r(M, 3 * D), r(M, D), r(M, F), r(M, F)
        y32, res32 = torch.empty(M, D, device=dev), r(M, D, dt=torch.float32)
        g_lp, ga = r(M, D), r(M, F)
        dW = {k: torch.zeros(*s, device=dev) for k, s in (("qkv", (3 * D, D)), ("p", (D, D)), ("1", (F, D)), ("2", (D, F)))}
        db = {k: torch.zeros(s, device=dev) for k, s in (("qkv", 3 * D), ("p", D), ("1", F), ("2", D))}
        e2 = 2

        def rep(name, t, nbytes, flops):
            if SELECT in name:
                report(name, t(), nbytes, flops)
        rep("fwd qkv [M,192]x[192,576]", lambda: timeit(lambda: ops.linear(x, w3, qkv, bias=b3), a.reps),
               M * D * e2 + M * 3 * D * e2, 2 * M * D * 3 * D)
        rep("fwd proj +res (f32 out)", lambda: timeit(lambda: ops.linear(o, wd, y32, bias=bd, epilogue=L.EPI_RESIDUAL,
                                                                   residual=res32, ld_residual=D), a.reps),
               M * D * e2 + 2 * M * D * 4, 2 * M * D * D)
        rep("fwd fc1 +GELU (act+pre)", lambda: timeit(lambda: ops.linear(x, w1, a_, bias=b1, epilogue=L.EPI_GELU, aux_out=pre,
                                                                    ld_aux_out=F), a.reps),
               M * D * e2 + 2 * M * F * e2, 2 * M * D * F)
        rep("fwd fc2 +res (K=768)", lambda: timeit(lambda: ops.linear(a_, w2, y32, bias=bd, epilogue=L.EPI_RESIDUAL,
                                                                 residual=res32, ld_residual=D), a.reps),
               M * F * e2 + 2 * M * D * 4, 2 * M * D * F)
        rep("bwd da = dx W2 * gelu'", lambda: timeit(lambda: ops.linear_dx(g_lp, w2, ga, epilogue=L.EPI_GELU_BWD, aux_in=pre,
                                                                      ld_aux_in=F), a.reps),
               M * D * e2 + 2 * M * F * e2, 2 * M * D * F)
        rep("bwd da = dx W2 * g (stored gelu')", lambda: timeit(lambda: ops.linear_dx(g_lp, w2, ga, epilogue=L.EPI_MUL_AUX,
                                                                               aux_in=pre, ld_aux_in=F), a.reps),
               M * D * e2 + 2 * M * F * e2, 2 * M * D * F)
        rep("fwd fc1 +GELU (act+gelu')", lambda: timeit(lambda: ops.linear(x, w1, a_, bias=b1, aux_out=pre, ld_aux_out=F,
                                                                      epilogue=L.EPI_GELU | L.EPI_GELU_GRAD), a.reps),
               M * D * e2 + 2 * M * F * e2, 2 * M * D * F)
        rep("bwd dh2 = da W1 (f32)", lambda: timeit(lambda: ops.linear_dx(ga, w1, y32), a.reps),
               M * F * e2 + M * D * 4, 2 * M * D * F)
        rep("bwd do = dy Wp", lambda: timeit(lambda: ops.linear_dx(g_lp, wd, o), a.reps), 2 * M * D * e2, 2 * M * D * D)
        rep("bwd dh1 = dqkv Wqkv (f32)", lambda: timeit(lambda: ops.linear_dx(qkv, w3, y32), a.reps),
               M * 3 * D * e2 + M * D * 4, 2 * M * D * 3 * D)
        rep("dW2 [192,768] (+db)", lambda: timeit(lambda: ops.linear_dw(g_lp, a_, dW["2"], db=db["2"]), a.reps),
               M * (D + F) * e2, 2 * M * D * F)
        rep("dW1 [768,192] (+db)", lambda: timeit(lambda: ops.linear_dw(ga, x, dW["1"], db=db["1"]), a.reps),
               M * (D + F) * e2, 2 * M * D * F)
        rep("dWp [192,192] (+db)", lambda: timeit(lambda: ops.linear_dw(g_lp, o, dW["p"], db=db["p"]), a.reps),
               M * 2 * D * e2, 2 * M * D * D)
        rep("dWqkv [576,192] (+db)", lambda: timeit(lambda: ops.linear_dw(qkv, x, dW["qkv"], db=db["qkv"]), a.reps),
               M * 4 * D * e2, 2 * M * D * 3 * D)
    if a.only == "base":
        # ViT-Base (C3) block products: D = 768, F = 3072, M = B x 1568
        Db, Fb = 768, 3072
        x, h = r(M, Db), r(M, Fb)
        wq, wp, w1, w2 = r(3 * Db, Db), r(Db, Db), r(Fb, Db), r(Db, Fb)
        bq, bd, b1 = r(3 * Db, dt=torch.float32), r(Db, dt=torch.float32), r(Fb, dt=torch.float32)
        qkv, a_, pre, o32 = r(M, 3 * Db), r(M, Fb), r(M, Fb), torch.empty(M, Db, device=dev)
        res = r(M, Db, dt=torch.float32)
        dWb = {k: torch.zeros(*s, device=dev) for k, s in (("qkv", (3 * Db, Db)), ("p", (Db, Db)), ("1", (Fb, Db)),
                                                           ("2", (Db, Fb)))}
        dbb = {k: torch.zeros(s, device=dev) for k, s in (("qkv", 3 * Db), ("p", Db), ("1", Fb), ("2", Db))}
        for name, fn, nb, fl in (
                ("base fwd qkv", lambda: ops.linear(x, wq, qkv, bias=bq), M * Db * 2 + M * 3 * Db * 2, 2 * M * Db * 3 * Db),
                ("base fwd proj +res", lambda: ops.linear(x, wp, o32, bias=bd, epilogue=L.EPI_RESIDUAL, residual=res,
                                                          ld_residual=Db), M * Db * 10, 2 * M * Db * Db),
                ("base fwd fc1 +GELU", lambda: ops.linear(x, w1, a_, bias=b1, epilogue=L.EPI_GELU, aux_out=pre,
                                                          ld_aux_out=Fb), M * Db * 2 + 2 * M * Fb * 2, 2 * M * Db * Fb),
                ("base fwd fc2 +res", lambda: ops.linear(h, w2, o32, bias=bd, epilogue=L.EPI_RESIDUAL, residual=res,
                                                         ld_residual=Db), M * Fb * 2 + M * Db * 8, 2 * M * Db * Fb),
                ("base dx da*gelu'", lambda: ops.linear_dx(x, w2, a_, epilogue=L.EPI_GELU_BWD, aux_in=pre, ld_aux_in=Fb),
                 M * Db * 2 + 2 * M * Fb * 2, 2 * M * Db * Fb),
                ("base dx dh2 (f32)", lambda: ops.linear_dx(h, w1, o32), M * Fb * 2 + M * Db * 4, 2 * M * Db * Fb),
                ("base dWqkv [2304,768]", lambda: ops.linear_dw(qkv, x, dWb["qkv"], db=dbb["qkv"]), M * 4 * Db * 2,
                 2 * M * Db * 3 * Db),
                ("base dWp [768,768]", lambda: ops.linear_dw(x, x, dWb["p"], db=dbb["p"]), M * 2 * Db * 2, 2 * M * Db * Db),
                ("base dW1 [3072,768]", lambda: ops.linear_dw(a_, x, dWb["1"], db=dbb["1"]), M * (Db + Fb) * 2,
                 2 * M * Db * Fb),
                ("base dW2 [768,3072]", lambda: ops.linear_dw(x, a_, dWb["2"], db=dbb["2"]), M * (Db + Fb) * 2,
                 2 * M * Db * Fb)):
            report(name, timeit(fn, a.reps), nb, fl)
    if a.only in ("", "copy"):
        # the chip's practical streaming rates on the same byte counts (torch's own kernels)
        src = torch.empty(M, F, dtype=bf, device=dev).normal_()
        dst = torch.empty_like(src)
        big = torch.empty(2 * M, F, dtype=bf, device=dev)
        report("copy 38.5 MB -> 38.5 MB (torch)", timeit(lambda: dst.copy_(src), a.reps), 2 * M * F * 2, 0)
        report("fill 77 MB (torch zero_)", timeit(lambda: big.zero_(), a.reps), 2 * M * F * 2, 0)
    if a.only in ("", "patch"):
        # patch embedding (C2: 16 clips of 16 x 3 x 224^2 -> 25,088 tokens x 192): im2col + row-slab GEMM
        # against the fused gather GEMM, with and without the bf16 cols side output (the dW operand)
        from oracle import cpu_ref
        px = torch.randn(B, 16, 3, 224, 224, device=dev)
        Kp = 1536
        wp = r(D, Kp)
        bp = torch.zeros(D, device=dev)
        pos = cpu_ref.sinusoid_table(N, D).to(dev)
        cols = torch.empty(M, Kp, dtype=bf, device=dev)
        x0 = torch.empty(M, D, device=dev)
        report("patch im2col (bf16 cols)", timeit(lambda: ops.patch_im2col(px, cols, 2, 16), a.reps), px.numel() * 6, 0)
        report("patch GEMM on cols (+bias+pos)", timeit(lambda: ops.linear(cols, wp, x0, bias=bp, epilogue=L.EPI_POS,
                                                                         pos=pos, pos_rows=N), a.reps),
               M * Kp * 2 + M * D * 4, 2 * M * D * Kp)
        report("patch fused gather GEMM", timeit(lambda: ops.patch_embed_fwd(px, wp, bp, pos, x0, 2, 16), a.reps),
               px.numel() * 4 + M * D * 4, 2 * M * D * Kp)
        report("patch fused gather GEMM + cols", timeit(lambda: ops.patch_embed_fwd(px, wp, bp, pos, x0, 2, 16,
                                                                                   cols=cols), a.reps),
               px.numel() * 6 + M * D * 4, 2 * M * D * Kp)
        dxp = r(M, D)
        dwp = torch.zeros(D, Kp, device=dev)
        dbp = torch.zeros(D, device=dev)
        nbp = ops.splitk_workspace_bytes(bf, D, Kp, M)
        wsp = torch.empty(nbp // 4 + 64, device=dev)
        report("patch dW (dx0^T cols, + db)", timeit(lambda: ops.linear_dw(dxp, cols, dwp, db=dbp, workspace=wsp), a.reps),
               M * (D + Kp) * 2 + D * Kp * 4, 2 * M * D * Kp)
    if a.only in ("", "attn"):
        Da = H * 64
        qkv = r(M, 3 * Da, dt=bf) * a.attn_scale
        o = torch.empty(M, Da, dtype=bf, device=dev)
        lse = torch.empty(B, H, N, device=dev)
        do = r(M, Da)
        dq = torch.empty(M, 3 * Da, dtype=bf, device=dev)
        ws = torch.empty(ops.attn_bwd_workspace_bytes(B, N, H) // 4 + 64, device=dev)
        f = 4.0 * B * H * N * N * 64
        done_f, done_b = set(), set()
        for v in [int(t, 0) for t in a.attn_variants.split(",")]:
            with L.knob("attn_variant", v):
                if (v & 15) not in done_f:
                    done_f.add(v & 15)
                    report(f"attn fwd [variant {v:#x}]", timeit(lambda: ops.attn_fwd(qkv, o, lse, B, N, H), a.reps),
                           M * 4 * Da * 2, f)
                if (v >> 4) not in done_b:
                    done_b.add(v >> 4)
                    if v >> 8:
                        print("  (bits 8 / 9: the dK/dV or the dQ pass skipped: timing only)")
                    report(f"attn bwd (rowprep+dkdv+dq) [variant {v:#x}]",
                           timeit(lambda: ops.attn_bwd(qkv, o, do, lse, dq, ws, B, N, H), a.reps), M * 8 * Da * 2,
                           2.5 * f)
    if a.only in ("", "linear"):
        # Linear plugin first layer at the real linear_video geometry (K = 120*128*128), f32, B = 4
        Bn, K, Nout = 4, 120 * 128 * 128, 256
        xf = torch.randn(Bn, K, device=dev)
        wf = torch.randn(Nout, K, device=dev) * K ** -0.5
        bf_ = torch.zeros(Nout, device=dev)
        yf = torch.zeros(Bn, Nout, device=dev)
        nb = ops.splitk_workspace_bytes(torch.float32, Bn, Nout, K)
        wsf = torch.empty(nb // 4 + 4, device=dev)
        report("linear_video L0 fwd (skinny f32)", timeit(lambda: ops.gemm(
            xf, wf, yf, M=Bn, N=Nout, K=K, a_kcontig=True, b_kcontig=True, lda=K, ldb=K, ldc=Nout,
            epilogue=L.EPI_ATOMIC | L.EPI_BIAS, bias=bf_, workspace=wsf), a.reps), (Bn + Nout) * K * 4, 2 * Bn * Nout * K)
        dyf = torch.randn(Bn, Nout, device=dev)
        dwf = torch.empty(Nout, K, device=dev)
        dbf = torch.zeros(Nout, device=dev)
        report("linear_video L0 dW (f32 stores)", timeit(lambda: ops.linear_dw(dyf, xf, dwf, db=dbf, accumulate=False),
                                                        a.reps), (Bn + Nout) * K * 4 + Bn * K * 4, 2 * Bn * Nout * K)
    if a.only in ("", "ln"):
        D = a.ln_dim
        x = r(M, D, dt=torch.float32)
        g, b = r(D, dt=torch.float32) + 1, r(D, dt=torch.float32)
        y = torch.empty(M, D, dtype=bf, device=dev)
        mu, rs = torch.empty(M, device=dev), torch.empty(M, device=dev)
        dx, dxl = torch.empty(M, D, device=dev), torch.empty(M, D, dtype=bf, device=dev)
        dg, dbb = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        report("ln fwd (f32 in, bf16 out)", timeit(lambda: ops.layernorm_fwd(x, g, b, 1e-12, y, mu, rs), a.reps),
               M * D * 6, 0)
        ops.layernorm_fwd(x, g, b, 1e-12, y, mu, rs)
        report("ln bwd (+dres, + bf16 copy)", timeit(lambda: ops.layernorm_bwd(x, x, mu, rs, g, dx, dg, dbb, dres=x,
                                                                               dx_lp=dxl), a.reps), M * D * 18, 0)
        dyl = y.clone()
        report("ln bwd (bf16 dy, +dres, + bf16 copy)", timeit(lambda: ops.layernorm_bwd(dyl, x, mu, rs, g, dx, dg, dbb,
                                                                                        dres=x, dx_lp=dxl), a.reps),
               M * D * 16, 0)
        xc = torch.empty_like(x)
        report("copy f32 (torch, read + write)", timeit(lambda: xc.copy_(x), a.reps), M * D * 8, 0)


if __name__ == "__main__":
    main()
