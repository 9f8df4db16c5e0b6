#!/bin/bash
# A/B builds of the attention kernels: libvspike_<name>.so = the in-tree objects with attention.hip
# (or another source) recompiled with extra flags.  usage: build_attn_variant.sh <name> <src.hip> [flags...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; src=$2; shift 2
B=video-spike_amd/vspike/_build
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I video-spike_amd/csrc -munsafe-fp-atomics"
OTHERS=$(ls $B/*.o | grep -v attention.o)
/opt/rocm/bin/hipcc $F "$@" -c "$src" -o /tmp/vs_var_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libvspike_$name.so $OTHERS /tmp/vs_var_$name.o
echo "built $B/libvspike_$name.so"
