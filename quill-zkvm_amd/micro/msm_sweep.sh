#!/bin/bash
# MSM check + profile on the GPU box: parity first, then a kernel trace, then
# timings per tuning setting (args: tag, then env settings).
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q \
  -k "msm or kzg or srs" --timeout 200 --timeout-method thread > gpurun_out/t_msm_$tag.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o msm \
  -- python3 quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 3 > gpurun_out/msm_prof_$tag.log 2>&1 || exit 1
for cfg in "$@"; do
  echo "== $cfg" >> gpurun_out/msm_sweep_$tag.log
  env $cfg timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 24 24,22 2 >> gpurun_out/msm_sweep_$tag.log 2>&1 || exit 1
done
