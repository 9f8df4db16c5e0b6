"""Host-side cost of the benched train step (C2, N=1): how long each phase of `Trainer.step` keeps
the Python thread busy WITHOUT waiting for the GPU, against the step's wall time.  A host time per
step close to the wall time means the GPU waits on the host (launch-bound), not on its kernels.

usage: python scripts/host_overhead.py [--steps 30] [--warmup 5]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "video-spike_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--model", default="vmae_tiny")
    ap.add_argument("--graph", action="store_true", help="also time the hipGraph-captured step")
    args = ap.parse_args()
    from vspike import VideoMAE, load_run_config
    from vspike.trainer import build_optimizer, Trainer
    cfg_dir = os.path.join(ROOT, "video-spike_amd", "config")
    config = load_run_config(os.path.join(cfg_dir, "model", args.model + ".yaml"),
                             os.path.join(cfg_dir, "train", "vmae_video.yaml"))
    config["model"]["decoder"]["output_dim"] = 100 * 128
    config["model"]["compute_dtype"] = "bf16"
    config["model"]["freeze_encoder"] = False
    dev = torch.device("cuda", 0)
    torch.manual_seed(1234)
    model = VideoMAE(config["model"]).to(dev)
    bb = model.backbone
    g = torch.Generator(device=dev).manual_seed(100)
    pixels = torch.randn(16, bb.num_frames, bb.num_channels, bb.image_size, bb.image_size, device=dev, generator=g)
    target = torch.poisson(torch.full((16, 100, 128), 0.3, device=dev), generator=g)
    opt, sched = build_optimizer(model, config, total_steps=10 * (args.steps + args.warmup) + 10)
    tr = Trainer(model, opt, sched, config=config)

    phases = {"forward": 0.0, "loss": 0.0, "backward": 0.0, "optimizer": 0.0, "scheduler": 0.0, "zero_grad": 0.0}

    def step_phased():
        t = time.perf_counter()
        out = model(pixels)
        t1 = time.perf_counter(); phases["forward"] += t1 - t
        loss = tr.criterion(out, target)
        t2 = time.perf_counter(); phases["loss"] += t2 - t1
        loss.backward()
        t3 = time.perf_counter(); phases["backward"] += t3 - t2
        opt.step()
        t4 = time.perf_counter(); phases["optimizer"] += t4 - t3
        sched.step()
        t5 = time.perf_counter(); phases["scheduler"] += t5 - t4
        opt.zero_grad(set_to_none=True)
        phases["zero_grad"] += time.perf_counter() - t5
        return loss.detach()

    for _ in range(args.warmup):
        tr.step(pixels, target)
    torch.cuda.synchronize()
    # 1) plain loop, as bench.py times it
    t0 = time.perf_counter()
    host = 0.0
    for _ in range(args.steps):
        a = time.perf_counter()
        tr.step(pixels, target)
        host += time.perf_counter() - a
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"loop: wall {wall / args.steps * 1e3:.3f} ms/step, host inside step() {host / args.steps * 1e3:.3f} ms/step")
    # 2) per-phase host time (the GPU keeps running behind)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_phased()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"phased: wall {wall / args.steps * 1e3:.3f} ms/step; host per phase (ms/step): " +
          ", ".join(f"{k} {v / args.steps * 1e3:.3f}" for k, v in phases.items()))
    # 3) host enqueue time with an idle GPU queue at the start of every step (upper bound of the
    #    launch cost: nothing can block on a full queue)
    hs = []
    for _ in range(args.steps):
        torch.cuda.synchronize()
        a = time.perf_counter()
        tr.step(pixels, target)
        hs.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    hs.sort()
    print(f"enqueue-only (GPU drained before each step): median {hs[len(hs) // 2] * 1e3:.3f} ms, "
          f"min {hs[0] * 1e3:.3f} ms")
    if args.graph:
        from vspike.graph import GraphedStep
        gs = GraphedStep(tr, pixels, target)
        for _ in range(3):
            gs.step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            gs.step()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"graph: wall {wall / args.steps * 1e3:.3f} ms/step")


if __name__ == "__main__":
    main()
