"""Instruction mix per basic block of one kernel in a hipcc -S listing (gfx950).

usage: python scripts/isa_mix.py <file.s> <kernel-name-substring>
Prints, for every basic block that issues MFMAs, the count of each instruction class and the
estimated issue cycles per MFMA-cycle (MI355X_MICROARCH.md 'vector-instruction ISSUE cost' row:
transcendental 8, other VALU 4, an MFMA holds vector issue for 8 of its 32 / 16 cycles).
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma_f32_32x32"):
        return "mfma32"
    if op.startswith("v_mfma_f32_16x16"):
        return "mfma16"
    if op.startswith(("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")):
        return "trans"
    if op.startswith("v_cvt_pk_bf16"):
        return "cvt_pk"
    if op.startswith("v_accvgpr"):
        return "accmov"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_"):
        return "ds_other"
    if op.startswith(("global_load_lds", "buffer_load") ) and "lds" in op:
        return "lds_dma"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


ISSUE = {"trans": 8, "valu": 4, "cvt_pk": 4, "accmov": 4, "ds_read": 4, "ds_other": 4, "lds_dma": 8,
         "vmem_load": 4, "vmem_store": 4, "mfma32": 8, "mfma16": 8, "nop": 4}


def main(path, name):
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*" + re.escape(name) + r"\w*:", l) or
                 (l.endswith(":") and name in l and not l.startswith(".")))
    blocks, cur, lab = OrderedDict(), Counter(), "entry"
    for l in lines[start + 1:]:
        if l.startswith("\t.end_amdhsa_kernel") or l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\w+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            blocks[lab] = cur
            cur, lab = Counter(), m.group(1)
            continue
        s = l.strip()
        if not s or s.startswith((";", ".")):
            continue
        op = s.split()[0]
        cur[classify(op)] += 1
        if op.startswith("s_cbranch") or op.startswith("s_branch"):
            cur["branch"] += 1
    blocks[lab] = cur
    for lab, c in blocks.items():
        mf = c["mfma32"] + c["mfma16"]
        if not mf:
            continue
        mcyc = 32 * c["mfma32"] + 16 * c["mfma16"]
        issue = sum(ISSUE.get(k, 1) * v for k, v in c.items() if k not in ("branch",))
        keys = ("mfma32", "mfma16", "trans", "cvt_pk", "valu", "accmov", "ds_read", "ds_other", "lds_dma", "vmem_load",
                "waitcnt", "barrier", "salu", "nop")
        print(f"{lab:14s} mfma-cyc {mcyc:5d} issue-cyc {issue:5d} ratio {issue / mcyc:4.2f}  " +
              " ".join(f"{k}={c[k]}" for k in keys if c[k]))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
