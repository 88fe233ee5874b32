#!/bin/bash
# MSM timings of library variants (micro/ab_<name>/libquill_gpu.so, "." = in-tree),
# alternating: the own-SRS 2^20 MSM (BASELINE config 2) and 2^24 on its SRS.
# usage: msm_own_lib_ab.sh <tag> <rounds> lib...
set -o pipefail
tag=$1; rounds=$2; shift 2
for i in $(seq "$rounds"); do
  for v in "$@"; do
    lib=quill-zkvm_amd/libquill_gpu.so; [ "$v" = "." ] || lib=quill-zkvm_amd/micro/ab_$v/libquill_gpu.so
    echo "== $v" >> gpurun_out/msm_own_lib_$tag.log
    MSM_PROF_OWN_SRS=1 QG_LIB=$lib timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 20 20 5 >> gpurun_out/msm_own_lib_$tag.log 2>&1 || exit 1
    QG_LIB=$lib timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 24 24 2 >> gpurun_out/msm_own_lib_$tag.log 2>&1 || exit 1
  done
done
