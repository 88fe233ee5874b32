#!/bin/bash
# NTT twiddles from the stage pyramid (default) vs the flat table (QG_NTT_FLAT=1):
# S-polynomial device time of MLEvalProof::prove at 2^k evaluations, alternating
set -o pipefail
k=${1:-23}
for r in 1 2; do
  for v in flat pyr; do
    e=""; [ "$v" = flat ] && e="QG_NTT_FLAT=1"
    printf '%s ' "$v"
    env $e timeout -k 10 200 python3 quill-zkvm_amd/micro/spoly_ab.py "$k" 1 || exit 1
  done
done
