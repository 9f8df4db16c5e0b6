"""Charged (algorithmic) bytes of every bench timer class vs the PMC HBM bytes of the kernels that
class launches (charged <= 1.05 x PMC, since PMC traffic below the algorithmic
bytes is impossible).

Two modes (scripts/pmc_bytes_check.sh runs them on the GPU box):
  run   <charged.json>            one ViT-Tiny block at the bench batch (128 clips, bf16, the bench's
                                  dispatch, weight-gradient products in order on the main stream), a
                                  warm-up step then one instrumented step; writes the libvspike timers'
                                  charged bytes and launch counts per class.  Run it under two
                                  rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).
  parse <pmc_dir> <charged.json> <out.json>
                                  walks the last step's dispatches in order, assigns each kernel to
                                  the timer class whose product launched it (the block executor's fixed
                                  order, csrc/vit_exec.hip), sums 2 x FETCH_SIZE + WRITE_SIZE (gfx950
                                  tallies a 128-B request of a 16-B/lane stream at 64 B:
                                  MI355X_MICROARCH.md "HBM") and compares.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# one block, forward then backward (serial side stream), with the kernel-name pattern that STARTS
# each class's run of dispatches; everything up to the next class's start belongs to the class
FWD = [("ln_fwd", r"ln_fwd_vec_kernel"), ("fwd_qkv", r"gemm_bf16_wres_kernel"), ("attn_fwd", r"attn_fwd_bf16_kernel"),
       ("fwd_proj", r"gemm_bf16_slab_kernel"), ("fwd_mlp", r"mlp_fwd_kernel")]
BWD = [("dx_mlp", r"mlp_bwd_da_kernel"), ("dw_fc2", r"gemm_dw_kernel"), ("dw_fc1", r"gemm_dw_kernel"),
       ("dx_fc1", r"gemm_bf16_slab_kernel"), ("dw_proj", r"gemm_dw_kernel"), ("dx_proj", r"gemm_bf16_slab_kernel"),
       ("attn_bwd", r"attn_rowprep_kernel"), ("dw_qkv", r"gemm_dw_kernel"), ("dx_qkv", r"gemm_bf16_slab_kernel")]

ONLY = {"fwd_mlp": r"mlp_fwd_kernel"}


def run(out):
    sys.path[:0] = [os.path.join(ROOT, "video-spike_amd"), ROOT]
    import torch
    from vspike import VideoMAE, FusedAdamW, poisson_nll_mean, ops, _lib as L
    conf = {"model_class": "VideoMAE", "freeze_encoder": False, "compute_dtype": "bf16",
            "backbone": {"hidden_size": 192, "num_attention_heads": 3, "intermediate_size": 768, "num_hidden_layers": 1},
            "encoder": {"output_dim": 64}, "decoder": {"output_dim": 12800}}
    torch.manual_seed(0)
    m = VideoMAE(conf).to("cuda")
    m.set_side_stream(False)
    B = 128
    px = torch.randn(B, 16, 3, 224, 224, device="cuda")
    y = torch.poisson(torch.full((B, 100, 128), 0.3, device="cuda"))
    opt = FusedAdamW([p for p in m.parameters() if p.requires_grad], lr=1e-6)

    def step():
        loss = poisson_nll_mean(m(px), y)
        loss.backward()
        opt.step()
        opt.zero_grad()
    step()
    torch.cuda.synchronize()
    ops.timing_enable((1 << len(L.TIMER_NAMES)) - 1)
    step()
    torch.cuda.synchronize()
    res = {}
    for tid, name in enumerate(L.TIMER_NAMES):
        n, ms, nbytes = ops.timing_collect(tid, with_bytes=True)
        if n:
            res[name] = {"launches": n, "charged_bytes_per_launch": nbytes / n, "ms_per_launch": ms / n}
    ops.timing_enable(0)
    json.dump(res, open(out, "w"), indent=1)


def _dispatches(d):
    rows = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = int(r.get("Dispatch_Id") or r.get("Dispatch_ID") or len(rows))
            ent = rows.setdefault(key, {"name": r["Kernel_Name"]})
            ent[r["Counter_Name"]] = ent.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"]) * 1024.0
    return [rows[k] for k in sorted(rows)]


def parse(pmc_dir, charged_json, out):
    charged = json.load(open(charged_json))
    fetch = _dispatches(os.path.join(pmc_dir, "FETCH_SIZE"))
    write = _dispatches(os.path.join(pmc_dir, "WRITE_SIZE"))
    assert [r["name"] for r in fetch] == [r["name"] for r in write], "the two passes dispatched differently"
    names = [r["name"] for r in fetch]
    nbytes = [2.0 * f.get("FETCH_SIZE", 0.0) + w.get("WRITE_SIZE", 0.0) for f, w in zip(fetch, write)]
    # the instrumented (last) step: from the last block-forward start
    starts = [i for i, n in enumerate(names) if re.search(FWD[0][1], n)]
    i = starts[-1]
    seq = FWD + BWD
    res = defaultdict(float)
    kern = defaultdict(list)
    for ci, (cls, pat) in enumerate(seq):
        while not re.search(pat, names[i]):
            i += 1
        j = i + 1
        nxt = seq[ci + 1][1] if ci + 1 < len(seq) else None
        # the class's own kernels: up to the next class start (the last class: its own pattern's kernels
        # plus their reduce / partial-sum launches, stopping at the first head / optimizer kernel)
        while j < len(names) and (nxt is None and re.search(r"ln_partsum|gemm_bf16_slab", names[j]) or
                                  nxt is not None and not re.search(nxt, names[j])):
            j += 1
        for k in range(i, j):
            # the block's last forward class is followed by the head's forward (casts, GEMMs, loss)
            # before the backward starts: count only the class's own kernel there
            if cls in ONLY and not re.search(ONLY[cls], names[k]):
                continue
            res[cls] += nbytes[k]
            kern[cls].append(names[k].split("(")[0])
        i = j
    rows = {}
    ok = True
    for cls, pmc in res.items():
        c = charged.get(cls, {}).get("charged_bytes_per_launch")
        if c is None:
            continue
        ratio = c / pmc if pmc else float("inf")
        good = ratio <= 1.05
        ok &= good
        rows[cls] = {"charged_bytes": round(c), "pmc_bytes": round(pmc), "charged_over_pmc": round(ratio, 3),
                     "ok": good, "kernels": kern[cls]}
        print(f"{cls:10s} charged {c / 1e6:9.1f} MB  PMC {pmc / 1e6:9.1f} MB  ratio {ratio:5.3f} {'ok' if good else 'OVER'}")
    json.dump({"method": "one ViT-Tiny block at 128 clips (bench dispatch, serial side stream), rocprofv3 --pmc "
                         "FETCH_SIZE / WRITE_SIZE in separate passes, traffic = 2 x FETCH_SIZE + WRITE_SIZE per "
                         "dispatch of the instrumented step; charged = libvspike timer bytes per launch",
               "all_ok": ok, "classes": rows}, open(out, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        parse(sys.argv[2], sys.argv[3], sys.argv[4])
