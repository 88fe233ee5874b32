#!/bin/bash
# HyperPlonk prove timings under env settings, alternating (same box):
# hp_env_ab.sh <tag> <rounds> ENV... ("-" = defaults)
set -o pipefail
tag=$1; rounds=$2; shift 2
for i in $(seq "$rounds"); do
  for cfg in "$@"; do
    e="$cfg"; [ "$cfg" = "-" ] && e=""
    echo "== $cfg" >> gpurun_out/hp_env_$tag.log
    env $e timeout -k 10 300 python3 quill-zkvm_amd/micro/hp_prof.py 20 3 >> gpurun_out/hp_env_$tag.log 2>&1 || exit 1
  done
done
