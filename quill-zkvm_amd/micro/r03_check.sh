#!/bin/bash
# Round-3 change check on the GPU box (arg: tag): the FP64-FMA multiplier
# microbenchmark, the sumcheck checks/timings/trace (sc_check.sh) and every
# sharded loopback test (world 2/4/8, generic expressions included).
#   gpurun -- 'bash quill-zkvm_amd/micro/r03_check.sh <tag>'
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 120 ./quill-zkvm_amd/micro/fp52_bench > gpurun_out/fp52_$tag.log 2>&1 || exit 1
bash quill-zkvm_amd/micro/sc_check.sh $tag || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 300 \
  --timeout-method thread > gpurun_out/t_multirank_$tag.log 2>&1 || exit 1
