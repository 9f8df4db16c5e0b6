"""HBM write / copy / read bandwidth with torch kernels (roofline calibration, debug aid)."""
import torch
def t(fn, reps=20):
    for _ in range(3): fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3
for mb in (38, 77, 256):
    n = mb * 2**20 // 2
    x = torch.empty(n, dtype=torch.bfloat16, device="cuda"); y = torch.empty_like(x)
    w = t(lambda: x.fill_(1.0)); c = t(lambda: y.copy_(x)); r = t(lambda: x.sum())
    print(f"{mb} MB: write {mb*2**20/w/1e12:.2f} TB/s  copy(r+w) {2*mb*2**20/c/1e12:.2f} TB/s  read(sum) {mb*2**20/r/1e12:.2f} TB/s")
