"""Where the CPU oracle's training step spends its time at B = 1 vs B = 4 (the
B = 4 backward / forward ratio of the bench's cpu_baseline was 9.6 on the GPU box vs ~3 at B = 1).

Runs oracle/cpu_ref.py's ViT-Tiny (C2) step on the CPU with torch.profiler: per batch, the forward
and the forward + backward wall time (median of `--reps` after a warm-up) and the top operators by
self CPU time of the fwd + bwd, plus the bytes of the attention probabilities autograd keeps for the
backward (B * H * N^2 f32 per layer).  Usage: python scripts/cpu_baseline_profile.py [--threads T]
"""
import argparse
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from oracle import cpu_ref, prng  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=os.cpu_count())
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batches", default="1,4")
    a = ap.parse_args()
    torch.set_num_threads(a.threads)
    cfg, n = cpu_ref.VIT_TINY, 128
    P = cpu_ref.to_torch(cpu_ref.make_vit_params(cfg, 64, n))
    px_all = torch.from_numpy(cpu_ref.make_pixels(cfg, 4))
    y_all = torch.from_numpy(prng.spike_targets(1, (4, 100, n)))
    N, H = cfg.num_tokens, cfg.num_attention_heads
    print(f"threads {a.threads}, ViT-Tiny (N = {N}, H = {H}, {cfg.num_hidden_layers} layers)")
    for B in [int(b) for b in a.batches.split(",")]:
        px, y = px_all[:B], y_all[:B]

        def fwd():
            with torch.no_grad():
                return cpu_ref.poisson_nll_mean(cpu_ref.videomae_plugin_forward(px, P, cfg, False), y)

        def fwd_bwd():
            loss = cpu_ref.poisson_nll_mean(cpu_ref.videomae_plugin_forward(px, P, cfg, False), y)
            loss.backward()
            for p in P.values():
                p.grad = None

        res = {}
        for name, fn in (("fwd", fwd), ("fwd_bwd", fwd_bwd)):
            fn()
            ts = []
            for _ in range(a.reps):
                t0 = time.perf_counter()
                fn()
                ts.append(time.perf_counter() - t0)
            res[name] = statistics.median(ts)
        probs = B * H * N * N * 4 * cfg.num_hidden_layers
        print(f"\nB={B}: fwd {res['fwd'] / B:.3f} s/clip, fwd+bwd {res['fwd_bwd'] / B:.3f} s/clip, "
              f"(fwd+bwd)/fwd {res['fwd_bwd'] / res['fwd']:.2f}; attention probabilities saved for the backward: "
              f"{probs / 1e9:.2f} GB ({B * H * N * N * 4 / 1e6:.0f} MB per layer)")
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            fwd_bwd()
        print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=12, max_name_column_width=40))


if __name__ == "__main__":
    main()
