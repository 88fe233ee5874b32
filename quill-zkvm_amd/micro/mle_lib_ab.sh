#!/bin/bash
# ML-PCS commit + open timings of library variants (micro/ab_<name>/libquill_gpu.so,
# "." = in-tree), alternating: mle_lib_ab.sh <tag> <rounds> lib...
set -o pipefail
tag=$1; rounds=$2; shift 2
for i in $(seq "$rounds"); do
  for v in "$@"; do
    lib=quill-zkvm_amd/libquill_gpu.so; [ "$v" = "." ] || lib=quill-zkvm_amd/micro/ab_$v/libquill_gpu.so
    printf '%s ' "$v" >> gpurun_out/mle_lib_$tag.log
    QG_LIB=$lib timeout -k 10 200 python3 quill-zkvm_amd/micro/mle_prof.py 22 8 >> gpurun_out/mle_lib_$tag.log 2>&1 || exit 1
  done
done
