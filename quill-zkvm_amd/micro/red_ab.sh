#!/bin/bash
# reduction A/B: MSM parity with the in-tree library, then kernel traces of the
# out-of-line (lib_ol) and inlined (lib_inl) combine builds
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q \
  -k "msm or kzg or commit" --timeout 200 --timeout-method thread > gpurun_out/t_red.log 2>&1 || exit 1
for v in ol inl; do
  QG_LIB=quill-zkvm_amd/micro/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/red_$v -o run -- \
    python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,22 3 > gpurun_out/red_$v.log 2>&1 || exit 1
  python3 profiles/kstats.py gpurun_out/red_$v > gpurun_out/red_$v.txt || exit 1
done
