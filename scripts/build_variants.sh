#!/bin/bash
# Build libvspike.so plus diagnostic variants in-tree; fails loudly.
#   libvspike_stamp.so : per-block cycle stamps (VS_STAMP) in attention + GEMM
set -euo pipefail
cd "$(dirname "$0")/.."
python - <<'PY'
import sys; sys.path.insert(0, 'video-spike_amd')
from vspike import build
build.build()
build.build(variant="stamp", defines=["VS_STAMP"])
PY
echo "built: $(ls video-spike_amd/vspike/_build/*.so | tr '\n' ' ')"
