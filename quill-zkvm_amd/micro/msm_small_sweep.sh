#!/bin/bash
# MSMs at 2^20 / 2^18 / 2^16 with their own SRS (window bits chosen per size),
# one line per chunk-length setting: msm_small_sweep.sh <tag> QG_MSM_ELOG=... ("-" = default)
set -o pipefail
tag=$1; shift
for cfg in "$@"; do
  e="$cfg"; [ "$cfg" = "-" ] && e=""
  echo "== $cfg" >> gpurun_out/msm_small_$tag.log
  env MSM_PROF_OWN_SRS=1 $e timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 20 20,18,16 3 >> gpurun_out/msm_small_$tag.log 2>&1 || exit 1
done
