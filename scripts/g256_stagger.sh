#!/bin/bash
# 256 x 256 GEMM: staggered start of the odd-slot workgroups (VSPIKE_G256_STAGGER x ~4 us), all
# g256-eligible C3 products forced onto the kernel
set -e
for st in 0 1 2 4 8; do
  echo "## stagger $st"
  VSPIKE_G256=1 VSPIKE_G256_STAGGER=$st timeout -k 10 120 python -u scripts/gemm_c3_bench.py --no-torch --only fwd | grep ours
  VSPIKE_G256=1 VSPIKE_G256_STAGGER=$st timeout -k 10 120 python -u scripts/gemm_c3_bench.py --no-torch --only dx | grep ours
done
