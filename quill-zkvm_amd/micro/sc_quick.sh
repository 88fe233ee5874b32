#!/bin/bash
# sumcheck change check on the GPU box (arg: tag): round digests at 2^20, the
# sumcheck / zero-check / HyperPlonk / generic GPU tests, two bench timings
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py \
  tests/test_gpu_hyperplonk.py tests/test_gpu_multirank.py tests/test_gpu_generic.py -m gpu -x -q \
  -k "sumcheck or zerocheck or hyperplonk or generic" --timeout 200 \
  --timeout-method thread > gpurun_out/t_sc_$tag.log 2>&1 || exit 1
timeout -k 10 60 ./quill-zkvm_amd/micro/sc_capi 20 50 > gpurun_out/sc_capi_$tag.log 2>&1 || exit 1
bash quill-zkvm_amd/micro/sc_ab.sh $tag base=- base2=- || exit 1
