#!/bin/bash
# S-polynomial device time of library variants (micro/ab_<name>/libquill_gpu.so,
# "." = in-tree), alternating: spoly_lib_ab.sh <tag> <log evals> <rounds> lib...
set -o pipefail
tag=$1; k=$2; rounds=$3; shift 3
for i in $(seq "$rounds"); do
  for v in "$@"; do
    lib=quill-zkvm_amd/libquill_gpu.so; [ "$v" = "." ] || lib=quill-zkvm_amd/micro/ab_$v/libquill_gpu.so
    printf '%s ' "$v" >> gpurun_out/spoly_lib_$tag.log
    QG_LIB=$lib timeout -k 10 200 python3 quill-zkvm_amd/micro/spoly_ab.py "$k" 1 >> gpurun_out/spoly_lib_$tag.log 2>&1 || exit 1
  done
done
