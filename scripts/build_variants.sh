#!/bin/bash
# Build libvspike.so plus diagnostic variants (stamp build) in-tree; fails loudly.
set -euo pipefail
cd "$(dirname "$0")/.."
python -c "import sys; sys.path.insert(0,'video-spike_amd'); from vspike import build; build.build()"
B=video-spike_amd/vspike/_build
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I video-spike_amd/csrc -munsafe-fp-atomics"
OTHERS=$(ls $B/*.o | grep -v attention.o | grep -v gemm.o)
/opt/rocm/bin/hipcc $F -DVS_STAMP -c video-spike_amd/csrc/attention.hip -o /tmp/vs_stamp_attention.o
/opt/rocm/bin/hipcc $F -DVS_STAMP -c video-spike_amd/csrc/gemm.hip -o /tmp/vs_stamp_gemm.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libvspike_stamp.so $OTHERS /tmp/vs_stamp_attention.o /tmp/vs_stamp_gemm.o
echo "built: $(ls $B/*.so | tr '\n' ' ')"
