#!/bin/bash
# one-shot-bases MSM at 2^24 by window bits (QG_MSM_WINDOW_BITS applies to every
# SRS the script builds): micro/oneshot_c_sweep.sh <out> c...
set -o pipefail
out=$1; shift
for c in "$@"; do
  printf 'c=%s ' "$c" >> "$out"
  QG_MSM_WINDOW_BITS=$c timeout -k 10 120 python3 -u quill-zkvm_amd/micro/oneshot_prof.py 24 5 >> "$out" 2>&1 || exit 1
done
