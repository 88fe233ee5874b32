#!/bin/bash
# FETCH_SIZE per random row gather at 8 / 16 / 32 GiB tables (TLB reach vs row bytes)
set -o pipefail
export TMPDIR=/tmp
for lr in 26 27 28; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/fcal_$lr -o p -f csv -- \
    python3 quill-zkvm_amd/micro/fetch_cal.py $lr 26 > gpurun_out/fcal_$lr.log 2>&1 || exit 1
done
