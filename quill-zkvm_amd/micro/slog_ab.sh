#!/bin/bash
# level-1 bucket weighted-sum width A/B (QG_MSM_SLOG1 = buckets per thread, log2)
set -o pipefail
export TMPDIR=/tmp
for s in 3 2 1 3 2; do
  QG_MSM_SLOG1=$s timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/sl_$s -o run -- \
    python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22,20 2 > gpurun_out/sl_$s.log 2>&1 || exit 1
  python3 profiles/kstats.py gpurun_out/sl_$s > gpurun_out/sl_$s.txt || exit 1
  echo "slog1=$s" >> gpurun_out/sl_all.txt; grep -E "k_msm_wsum|k_msm_combine" gpurun_out/sl_$s.txt >> gpurun_out/sl_all.txt
done
