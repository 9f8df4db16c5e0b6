#!/bin/bash
# PMC passes over the fc1 + GELU product on the W-resident kernel and on the whole-K tile kernel.
export TMPDIR=/tmp
ONLY="gemm:fwd fc1" timeout -k 10 400 scripts/pmc_attn.sh gpurun_out/pmc_wres > gpurun_out/pmc_wres.log 2>&1 || exit $?
VSPIKE_NO_WRES=1 ONLY="gemm:fwd fc1" timeout -k 10 400 scripts/pmc_attn.sh gpurun_out/pmc_fullk > gpurun_out/pmc_fullk.log 2>&1 || exit $?
python3 scripts/pmc_json.py gpurun_out/pmc_wres gpurun_out/pmc_wres.json gemm_bf16 && python3 scripts/pmc_json.py gpurun_out/pmc_fullk gpurun_out/pmc_fullk.json gemm_bf16
python3 - <<'PY'
import json
for f in ("gpurun_out/pmc_wres.json", "gpurun_out/pmc_fullk.json"):
    d = json.load(open(f))
    for k, v in d["kernels"].items():
        c = v["counters"]
        print(f, k[:50], {x: round(v[x], 3) for x in v if x.endswith("frac")}, "cyc", round(v.get("kernel_cycles", 0)),
              {x: c.get(x) for x in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD",
                                      "SQ_INSTS_VALU_TRANS_F32", "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES")},
              "hbm", v.get("hbm_bytes"))
PY
