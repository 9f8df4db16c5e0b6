#!/bin/bash
# A/B timing of attention builds: scripts/ab_attn.sh name1 name2 ...  ("main" = libvspike.so)
B=$PWD/video-spike_amd/vspike/_build
for n in "$@"; do
  if [ "$n" = main ]; then lib=$B/libvspike.so; else lib=$B/libvspike_$n.so; fi
  echo "== $n"; VSPIKE_LIB=$lib timeout -k 10 120 python scripts/microbench.py --only attn --reps 50 2>&1 | grep attn || exit 1
done
