#!/bin/bash
# MSM bucketing / accumulation overlap A/B (QG_MSM_PIPE settings), alternating
# rounds on one box: msm_pipe_ab.sh <tag> <log_max> <sizes> <reps> <rounds> CFG...
# (CFG: space-separated env assignments in one argument, "-" = defaults)
set -o pipefail
tag=$1; lmax=$2; sizes=$3; reps=$4; rounds=$5; shift 5
for i in $(seq "$rounds"); do
  for cfg in "$@"; do
    e="$cfg"; [ "$cfg" = "-" ] && e=""
    echo "== $cfg" >> gpurun_out/msm_pipe_$tag.log
    env $e timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py "$lmax" "$sizes" "$reps" >> gpurun_out/msm_pipe_$tag.log 2>&1 || exit 1
  done
done
