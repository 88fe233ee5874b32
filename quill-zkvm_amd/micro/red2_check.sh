#!/bin/bash
# bucket-reduction rewrite check (arg: tag): MSM / KZG parity, then MSM
# timings at 2^24 / 2^22 / 2^20 for several accumulation round counts and the
# old 128-entry chunks, and one kernel trace
#   gpurun -- 'bash quill-zkvm_amd/micro/red2_check.sh <tag>'
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_multirank.py \
  -m gpu -x -v -k "msm or kzg or commit or mle_open" --timeout 200 --timeout-method thread > gpurun_out/t_red2_$tag.log 2>&1 || exit 1
for r in 2 1 3; do
  QG_MSM_ROUNDS=$r timeout -k 10 200 python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 5 > gpurun_out/red2_${tag}_r$r.log 2>&1 || exit 1
done
QG_MSM_Q4=0 timeout -k 10 200 python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 5 > gpurun_out/red2_${tag}_noq4.log 2>&1 || exit 1
QG_MSM_ELOG=7 timeout -k 10 200 python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 5 > gpurun_out/red2_${tag}_e7.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/red2_$tag -o run -- \
  python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 3 > gpurun_out/red2_${tag}_prof.log 2>&1 || exit 1
python3 profiles/kstats.py gpurun_out/red2_$tag > gpurun_out/red2_$tag.txt || exit 1
