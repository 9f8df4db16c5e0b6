"""Scan hipcc -S listings (gfx950) for the store-data hazard the fused MLP backward hit: a
buffer_store_dwordx2/x3/x4 whose soffset is an SGPR, followed IMMEDIATELY by a VALU instruction
that writes one of the store's data VGPRs (measured on MI355X: the store then wrote the VALU's new
value into dwords 1.. of lanes 12-15 of every 16; hipcc inserted no wait state).

usage: python scripts/check_store_hazard.py [file.hip ...]   (default: every csrc/*.hip)
Compiles each file to device assembly in a temp dir and prints every hazardous pair; exit 1 if any.
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "video-spike_amd", "csrc")


def regs(op):
    out = set()
    for m in re.finditer(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b", op):
        if m.group(3):
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def scan(asm_path):
    hits = []
    lines = [l.strip() for l in open(asm_path)]
    func = "?"
    prev = None  # (data regs, line) of a store with an SGPR soffset
    for i, t in enumerate(lines):
        if re.match(r"^_Z\w+:", t):
            func = t[:-1]
        if not t or t.startswith((";", ".")):
            continue
        parts = t.split(None, 1)
        op = parts[0]
        args = [a.strip() for a in parts[1].split(",")] if len(parts) > 1 else []
        if prev is not None and op.startswith("v_") and args:
            if regs(args[0]) & prev[0]:
                hits.append((func, prev[1], t))
        prev = None
        if re.match(r"buffer_store_dwordx[234]$", op) and len(args) >= 4 and args[3].startswith("s"):
            prev = (regs(args[0]), t)
    return hits


def main(files):
    files = files or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for f in files:
            out = os.path.join(td, os.path.basename(f) + ".s")
            cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S",
                   "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-munsafe-fp-atomics", f, "-o", out]
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                print(f"{os.path.basename(f)}: compile failed\n{r.stderr[-2000:]}")
                bad += 1
                continue
            hits = scan(out)
            for func, st, v in hits:
                print(f"{os.path.basename(f)}: {func[:60]}: {st}  ->  {v}")
            bad += len(hits)
            print(f"{os.path.basename(f)}: {len(hits)} hazardous store / VALU pairs", file=sys.stderr)
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
