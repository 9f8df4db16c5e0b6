#!/bin/bash
# A/B builds: libvspike_<name>.so = the in-tree objects with <obj> replaced by <src.hip> compiled with
# extra flags.  usage: build_variant.sh <name> <obj, e.g. norm.o> <src.hip> [flags...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; obj=$2; src=$3; shift 3
B=video-spike_amd/vspike/_build
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -I include -I video-spike_amd/csrc -munsafe-fp-atomics"
OTHERS=$(ls $B/*.o | grep -v "/$obj\$")
/opt/rocm/bin/hipcc $F "$@" -c "$src" -o /tmp/vs_var_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/libvspike_$name.so $OTHERS /tmp/vs_var_$name.o -lpthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo "built $B/libvspike_$name.so"
