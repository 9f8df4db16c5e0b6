"""Diagnostic: the R3D plugin's gradients at C4 geometry (32 x 112 x 112, B = 2) vs the f64 oracle,
per parameter, and bitwise repeatability of two GPU runs.  usage: python scripts/dbg/r3d_grad_check.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import cpu_ref, prng  # noqa: E402


def main():
    from vspike import R3D, poisson_nll_mean
    T, S, B, n = 32, 112, 2, 256
    cfg = cpu_ref.R3DCfg(num_frames=T, image_size=S)
    params = cpu_ref.make_r3d_params(cfg, 64, n)
    P = {k: torch.from_numpy(v).double().requires_grad_() for k, v in params.items()}
    px = torch.from_numpy(cpu_ref.make_r3d_pixels(cfg, B, seed=5))
    y = torch.from_numpy(prng.spike_targets(5, (B, 100, n)))
    running = {}
    for name, ci, co, *_ in cpu_ref.r3d_conv_specs(cfg):
        bn = name[:-2] + ".1"
        running[bn + ".running_mean"] = torch.zeros(co, dtype=torch.float64)
        running[bn + ".running_var"] = torch.ones(co, dtype=torch.float64)
    ref = cpu_ref.r3d18_forward(px.double(), P, cfg, running=running)
    cpu_ref.poisson_nll_mean(ref, y.double()).backward()
    conf = {"model_class": "R3D", "compute_dtype": "fp32", "freeze_encoder": False,
            "backbone": {"num_frames": T, "image_size": S, "num_channels": 3},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 100 * n}}
    runs = []
    for rep in range(2):
        m = R3D(conf).to("cuda")
        m.load_reference_state_dict({k: torch.from_numpy(v) for k, v in params.items()}, strict=False)
        out = m(px.to("cuda"))
        if rep == 0:
            print("log-rates maxrel", float((out.detach().double().cpu() - ref.detach()).abs().max() / ref.abs().max()))
            sd = m.reference_state_dict()
            for k in running:
                if "layer4" in k or "stem" in k or "layer3.1" in k:
                    # running = 0.9 init + 0.1 batch stat: compare the batch statistic itself
                    init = 0.0 if k.endswith("mean") else 1.0
                    gb, rb = (sd[k].double().cpu() - 0.9 * init) / 0.1, (running[k] - 0.9 * init) / 0.1
                    print(f"  {k:36s} batch stat maxrel {float((gb - rb).abs().max() / rb.abs().max()):.2e}")
        loss = poisson_nll_mean(out, y.to("cuda"))
        loss.backward()
        torch.cuda.synchronize()
        runs.append((m, m.enc_flat.grad.detach().clone()))
    m, g = runs[0]
    print("bitwise repeat:", torch.equal(runs[0][1], runs[1][1]))
    lay = m.layout
    for c in lay.convs:
        gw = lay.enc.view(g, c.name + ".weight")[..., :c.ci_ref].permute(0, 4, 1, 2, 3).double().cpu()
        rw = P[c.name + ".weight"].grad
        bn = c.name[:-2] + ".1"
        gb = lay.enc.view(g, bn + ".bias").double().cpu()
        rb = P[bn + ".bias"].grad
        gg = lay.enc.view(g, bn + ".weight").double().cpu()
        rg = P[bn + ".weight"].grad
        print(f"{c.name:24s} dW {float((gw - rw).norm() / rw.norm()):.2e}  dgamma {float((gg - rg).norm() / rg.norm()):.2e}"
              f"  dbeta {float((gb - rb).norm() / rb.norm()):.2e}")


if __name__ == "__main__":
    main()
