#!/bin/bash
# round-5 A/B step: parity subset on the in-tree library, then MSM and
# HyperPlonk timings of micro/ab_base (HEAD build) vs the in-tree library,
# alternating.  usage: r05_ab.sh <tag> [rounds]
set -o pipefail
tag=$1; rounds=${2:-2}
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_altpaths.py \
  tests/test_gpu_hyperplonk.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
bash quill-zkvm_amd/micro/msm_lib_ab.sh $tag $rounds base . || exit 1
bash quill-zkvm_amd/micro/hp_lib_ab.sh $tag $rounds base . || exit 1
cat gpurun_out/msm_lib_$tag.log gpurun_out/hp_lib_$tag.log
