#!/bin/bash
# MSM timings under env settings, alternating rounds (same box):
# msm_env_ab.sh <tag> <log_max> <sizes> <rounds> ENV... ("-" = defaults)
set -o pipefail
tag=$1; lmax=$2; sizes=$3; rounds=$4; shift 4
for i in $(seq "$rounds"); do
  for cfg in "$@"; do
    e="$cfg"; [ "$cfg" = "-" ] && e=""
    echo "== $cfg" >> gpurun_out/msm_env_$tag.log
    env $e timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py "$lmax" "$sizes" 2 >> gpurun_out/msm_env_$tag.log 2>&1 || exit 1
  done
done
