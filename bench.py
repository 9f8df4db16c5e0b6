"""Benchmark: clips/sec of the full video->spike TRAIN step (BASELINE config C2 at N=1).

Workload (BASELINE.json configs[1]): ViT-Tiny/16 encoder (d192, 3 heads, 12 layers, tubelet 2)
on 16x224x224 clips (1568 tokens) -> Linear(1568*192 -> 64) -> Linear(64 -> 100*128) log-rates,
PoissonNLL mean, full backward INCLUDING the encoder (freeze_encoder: false), fused AdamW +
OneCycleLR step, bf16 compute / f32 accumulate, batch 16 clips per GPU, synthetic data
(random pixels, Poisson spike targets) resident in HBM.  One process per GPU; for N > 1 each
rank trains its own 16 clips and gradients are all-reduced over RCCL (weak scaling).

Prints ONE JSON line (rank 0).  `roofline` is measured live with hipEvents bracketing every
attention launch on its own stream inside the timed region; `cpu_baseline` times the CPU fp32
oracle (oracle/cpu_ref.py, a torch-CPU restatement of the same step) on the host cores.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "video-spike_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=16, help="clips per GPU")
    ap.add_argument("--neurons", type=int, default=128)
    ap.add_argument("--model", default="vmae_tiny", help="config/model/<name>.yaml")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the CPU-oracle baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timers", action="store_true", help="do not bracket kernels with hipEvents")
    return ap.parse_args()


def cpu_baseline(model_cfg, neurons, seconds):
    """Oracle (torch-CPU fp32 restatement) train step fwd+bwd on batch-1 clips, bounded in time."""
    from oracle import cpu_ref, prng
    bb = model_cfg["backbone"]
    cfg = cpu_ref.ViTCfg(**{k: (float(v) if k == "layer_norm_eps" else int(v)) for k, v in bb.items()})
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, neurons))
    px = torch.from_numpy(cpu_ref.make_pixels(cfg, 1))
    y = torch.from_numpy(prng.spike_targets(1, (1, 100, neurons)))
    threads = torch.get_num_threads()
    n, t0 = 0, time.perf_counter()
    while True:
        loss = cpu_ref.poisson_nll_mean(cpu_ref.videomae_plugin_forward(px, P, cfg, freeze_encoder=False), y)
        loss.backward()
        for p in P.values():
            p.grad = None
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds or (n >= 2 and el * (n + 1) / n > 2 * seconds):
            break
    return {"value": n / el, "unit": "clips/sec", "cores": threads, "kind": "port",
            "sample": f"{n} clips x fwd+bwd (ViT-Tiny/16 encoder trainable + head + PoissonNLL), batch 1, "
                      f"fp32 torch-CPU oracle, {el:.1f} s"}


def _traffic(op):
    """HBM bytes per launch of `op` from the committed PMC summary (scripts/pmc_traffic.sh: separate
    FETCH_SIZE / WRITE_SIZE passes, FETCH doubled per the gfx950 correction), or None."""
    import glob as _glob
    files = sorted(_glob.glob(os.path.join(ROOT, "profiles", "*_traffic.json")))
    if not files:
        return None
    try:
        d = json.load(open(files[-1]))
        return round(d["ops"][op]["traffic_bytes"], 0)
    except (KeyError, ValueError, OSError):
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    from vspike import VideoMAE, load_run_config, ops, poisson_nll_mean
    from vspike import _lib as L
    from vspike.dp import GradExchange
    from vspike.trainer import build_optimizer, Trainer

    cfg_dir = os.path.join(ROOT, "video-spike_amd", "config")
    config = load_run_config(os.path.join(cfg_dir, "model", args.model + ".yaml"),
                             os.path.join(cfg_dir, "train", "vmae_video.yaml"))
    config["model"]["decoder"]["output_dim"] = 100 * args.neurons       # src/train.py:41
    config["model"]["compute_dtype"] = args.dtype
    config["model"]["freeze_encoder"] = False
    torch.manual_seed(1234 + rank)
    model = VideoMAE(config["model"]).to(dev)
    bb = model.backbone
    B = args.batch
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    pixels = torch.randn(B, bb.num_frames, bb.num_channels, bb.image_size, bb.image_size, device=dev, generator=g)
    lam = torch.exp(torch.randn(B, 100, args.neurons, device=dev, generator=g) - 2.0).clamp(0.01, 5.0)
    target = torch.poisson(lam, generator=g)
    total = args.warmup + args.steps
    opt, sched = build_optimizer(model, config, total_steps=total, world=world)
    exchange = GradExchange(model) if world > 1 else None
    trainer = Trainer(model, opt, sched, criterion=poisson_nll_mean, exchange=exchange)

    for _ in range(args.warmup):
        trainer.step(pixels, target)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    timers = 0 if args.no_timers else (1 << L.TIMER_ATTN_FWD) | (1 << L.TIMER_ATTN_BWD)
    ops.timing_enable(timers)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    losses = []
    for _ in range(args.steps):
        losses.append(trainer.step(pixels, target))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern = {}
    for name, tid in (("attn_fwd", L.TIMER_ATTN_FWD), ("attn_bwd", L.TIMER_ATTN_BWD)):
        n, ms = ops.timing_collect(tid) if timers else (0, 0.0)
        kern[name] = (n, ms)
    ops.timing_enable(0)
    if world > 1:
        t = torch.tensor([elapsed], device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(losses[-1].item())

    clips = world * B * args.steps
    value = clips / elapsed
    N, H, Lyr = bb.num_tokens, bb.num_attention_heads, bb.num_hidden_layers
    fwd_flop = 4.0 * B * H * N * N * 64                 # QK^T + PV per launch (one layer)
    per = {"attn_fwd": fwd_flop, "attn_bwd": 2.5 * fwd_flop}
    roof_all = {}
    for k, (n, ms) in kern.items():
        if n:
            avg_s = ms / n / 1e3
            ach = per[k] / avg_s / 1e12
            roof_all[k] = {"launches": n, "avg_ms": ms / n, "flop_per_launch": per[k], "achieved_tflops": ach}
    dom = max(roof_all, key=lambda k: roof_all[k]["avg_ms"] * roof_all[k]["launches"]) if roof_all else None
    peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
    roofline = None
    if dom:
        r = roof_all[dom]
        roofline = {"bound": "mfma", "kernel": dom, "achieved": round(r["achieved_tflops"], 2), "peak": peak,
                    "unit": "TFLOP/s", "frac": round(r["achieved_tflops"] / peak, 4), "traffic": _traffic(dom),
                    "avg_launch_ms": round(r["avg_ms"], 4), "flop_per_launch": r["flop_per_launch"],
                    "all": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                            for k, v in roof_all.items()}}
    # algorithmic train FLOPs per clip (BASELINE.md convention: train = 3 x forward)
    D, F, K = bb.hidden_size, bb.intermediate_size, bb.patch_dim
    fwd_clip = Lyr * (2 * N * D * 3 * D + 2 * N * D * D + 4 * N * D * F + 4 * N * N * D) + 2 * N * K * D \
        + 2 * N * D * 64 + 2 * 64 * 100 * args.neurons
    step_tflops = 3 * fwd_clip * B * world * args.steps / elapsed / 1e12

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(config["model"], args.neurons, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": "clips/sec (16-frame 224x224) train step", "value": round(value, 3), "unit": "clips/sec",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": args.dtype, "data": "synthetic (randn pixels, Poisson targets), random-init",
            "config": {"workload": "C2 ViT-Tiny/16 16x224x224 -> 128 neurons, encoder+head fwd+bwd+AdamW",
                       "model": args.model, "global_batch": B * world, "clips_per_gpu": B, "seq_len": N,
                       "parallelism": f"dp{world}"},
            "mfma_util_pct": round(100.0 * step_tflops / peak, 2),
            "model_tflops": round(step_tflops, 2),
            "roofline": roofline, "cpu_baseline": cpu, "final_loss": round(final_loss, 6),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
