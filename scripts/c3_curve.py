"""Loss trajectory of the bench's synthetic C3 (ViT-Base, 512 neurons) setup in fp32 and bf16:
shows whether a divergence is a property of the setup (both dtypes) or of the bf16 kernels.
usage: python scripts/c3_curve.py [steps] [--freeze]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "video-spike_amd"))
import torch  # noqa: E402

from vspike import VideoMAE, load_run_config, poisson_nll_mean  # noqa: E402
from vspike.trainer import Trainer, build_optimizer  # noqa: E402


def curve(dtype, steps, freeze, model="vmae_video", neurons=512, B=8, lr=None):
    cfg_dir = os.path.join(ROOT, "video-spike_amd", "config")
    config = load_run_config(os.path.join(cfg_dir, "model", model + ".yaml"),
                             os.path.join(cfg_dir, "train", "vmae_video.yaml"))
    config["model"]["decoder"]["output_dim"] = 100 * neurons
    config["model"]["compute_dtype"] = dtype
    config["model"]["freeze_encoder"] = freeze
    if lr is not None:
        config["optimizer"]["lr"] = lr
    torch.manual_seed(1234)
    m = VideoMAE(config["model"]).cuda()
    bb = m.backbone
    g = torch.Generator(device="cuda").manual_seed(100)
    px = torch.randn(B, bb.num_frames, bb.num_channels, bb.image_size, bb.image_size, device="cuda", generator=g)
    lam = torch.exp(torch.randn(B, 100, neurons, device="cuda", generator=g) - 2.0).clamp(0.01, 5.0)
    y = torch.poisson(lam, generator=g)
    opt, sched = build_optimizer(m, config, total_steps=steps)
    tr = Trainer(m, opt, sched, criterion=poisson_nll_mean)
    out = []
    for _ in range(steps):
        out.append(float(tr.step(px, y)))
    with torch.no_grad():
        lr = m(px)
    return out, float(lr.abs().max())


if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    freeze = "--freeze" in sys.argv
    model = "vmae_tiny" if "--tiny" in sys.argv else "vmae_video"
    lr = float(sys.argv[sys.argv.index("--lr") + 1]) if "--lr" in sys.argv else None
    for dt in ("fp32", "bf16"):
        c, mx = curve(dt, steps, freeze, model=model, neurons=128 if model == "vmae_tiny" else 512, lr=lr)
        print(dt, "losses", " ".join(f"{v:.4g}" for v in c), "| max |log-rate| after:", f"{mx:.4g}", flush=True)
