#!/bin/bash
# window-size A/B at 2^24: kernel traces of one SRS + 3 MSMs at c = 20 and c = 22
set -o pipefail
export TMPDIR=/tmp
for c in 20 22; do
  QG_MSM_WINDOW_BITS=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/win_$c -o run -- \
    python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24 3 > gpurun_out/win_$c.log 2>&1 || exit 1
  python3 profiles/kstats.py gpurun_out/win_$c > gpurun_out/win_$c.txt || exit 1
done
