#!/bin/bash
# MSM parity + window sweep at SRS 2^22 / 2^20 (arg: tag)
set -o pipefail
export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q \
  -k "msm or kzg or srs or mle" --timeout 200 --timeout-method thread > gpurun_out/t_msm_$tag.log 2>&1 || exit 1
for c in 17 19 20; do
  echo "== c=$c" >> gpurun_out/msm_sweep2_$tag.log
  QG_MSM_WINDOW_BITS=$c timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 22 22,20 3 >> gpurun_out/msm_sweep2_$tag.log 2>&1 || exit 1
done
timeout -k 10 200 python3 quill-zkvm_amd/micro/msm_prof.py 24 24 3 >> gpurun_out/msm_sweep2_$tag.log 2>&1
