"""HBM write-only and copy rates on one MI355X (the ceiling for store-bound products such as the
fc1 forward, which writes 8x what it reads).  hipEvents around back-to-back launches of torch's own
fill / copy kernels over 1 GiB buffers.  Usage: python scripts/store_rate.py"""
import torch


def rate(fn, nbytes, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = 1e3 * s.elapsed_time(e) / reps
    return us, nbytes / us / 1e6


def main():
    n = 1 << 30
    a = torch.empty(n // 2, dtype=torch.bfloat16, device="cuda")
    b = torch.empty_like(a)
    a.fill_(1.0)
    for name, fn, nb in [("write-only (fill_)", lambda: b.fill_(2.0), n),
                         ("copy 1:1 (copy_)", lambda: b.copy_(a), 2 * n)]:
        us, tb = rate(fn, nb)
        print(f"{name:22s} {us:8.1f} us  {tb:5.2f} TB/s over {nb / 1e9:.2f} GB")


if __name__ == "__main__":
    main()
