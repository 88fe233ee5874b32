#!/bin/bash
# bucket-reduction A/B (arg: tag): MSM timings at 2^24 / 2^20 per env variant
#   gpurun -- 'bash quill-zkvm_amd/micro/red3_ab.sh <tag> "NAME=V NAME=V" ...'
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  echo "== $spec" >> gpurun_out/red3_$tag.log
  env $spec timeout -k 10 200 python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 5 >> gpurun_out/red3_$tag.log 2>&1 || exit 1
  i=$((i+1))
done
