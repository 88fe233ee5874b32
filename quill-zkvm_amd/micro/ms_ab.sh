#!/bin/bash
# accumulate A/B of two library builds (lib_head = HEAD, lib_new = working tree):
# MSM parity with the in-tree library, then alternating 2^24 kernel traces
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q \
  -k "msm or kzg or commit" --timeout 200 --timeout-method thread > gpurun_out/t_ms.log 2>&1 || exit 1
for r in 1 2; do
  for v in head new; do
    QG_LIB=quill-zkvm_amd/micro/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ms_${v}_$r -o run -- \
      python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24 3 > gpurun_out/ms_${v}_$r.log 2>&1 || exit 1
    python3 profiles/kstats.py gpurun_out/ms_${v}_$r > gpurun_out/ms_${v}_$r.txt || exit 1
  done
done
