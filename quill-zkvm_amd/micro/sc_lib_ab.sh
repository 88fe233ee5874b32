#!/bin/bash
# sumcheck C-ABI timing of library variants (micro/ab_<name>/libquill_gpu.so,
# "." = the in-tree build), alternating: sc_lib_ab.sh <nv> <steps> <rounds> lib...
set -o pipefail
cd "$(dirname "$0")/.."
nv=$1; steps=$2; rounds=$3; shift 3
for i in $(seq "$rounds"); do
  for v in "$@"; do
    d=$v; [ "$v" = "." ] || d=micro/ab_$v
    printf '%s ' "$v"
    LD_LIBRARY_PATH=$d timeout -k 5 60 micro/sc_capi "$nv" "$steps" || exit 1
  done
done
