#!/bin/bash
# radix-4 vs radix-2 NTT passes: S-polynomial device time of MLEvalProof::prove
# at 2^k evaluations (one context), alternating QG_NTT_R2=1 / default
set -o pipefail
k=${1:-23}
for r in 1 2; do
  for v in r2 r4; do
    e=""; [ "$v" = r2 ] && e="QG_NTT_R2=1"
    printf '%s ' "$v"
    env $e timeout -k 10 200 python3 quill-zkvm_amd/micro/spoly_ab.py "$k" 1 || exit 1
  done
done
