#!/bin/bash
# reduction rewrite check (arg: tag): MSM/KZG/ML-open parity, then A/B timings
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_multirank.py \
  -m gpu -x -q -k "msm or kzg or commit or mle_open" --timeout 200 --timeout-method thread > gpurun_out/t_red4_$tag.log 2>&1 || exit 1
bash quill-zkvm_amd/micro/red3_ab.sh $tag "$@" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/red4_$tag -o run -- \
  python3 -u quill-zkvm_amd/micro/msm_prof.py 24 24,20 3 > gpurun_out/red4_${tag}_prof.log 2>&1 || exit 1
python3 profiles/kstats.py gpurun_out/red4_$tag msm > gpurun_out/red4_$tag.txt || exit 1
