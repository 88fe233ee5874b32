#!/bin/bash
# MSM timings per tuning setting only (args: tag, then env settings, e.g. QG_MSM_ELOG=7)
set -o pipefail
tag=$1; shift
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/msm_sweep_$tag.log
  env $cfg timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 2 >> gpurun_out/msm_sweep_$tag.log 2>&1 || exit 1
done
