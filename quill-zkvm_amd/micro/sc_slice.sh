#!/bin/bash
# slice-tail check on the GPU box (arg: tag): digests, sumcheck tests, C-ABI
# timing for the slice tail and the streaming tail, bench, phase trace
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}.log 2>&1 || exit 1
timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 13 >> gpurun_out/sc_dig_${tag}.log 2>&1 || exit 1
QG_SC_OLD_TAIL=1 timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 13 >> gpurun_out/sc_dig_${tag}.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py \
  tests/test_gpu_hyperplonk.py tests/test_gpu_multirank.py tests/test_gpu_generic.py -m gpu -x -q \
  -k "sumcheck or zerocheck or hyperplonk or generic" --timeout 200 \
  --timeout-method thread > gpurun_out/t_sc_$tag.log 2>&1 || exit 1
timeout -k 10 60 ./quill-zkvm_amd/micro/sc_capi 20 50 > gpurun_out/sc_capi_$tag.log 2>&1 || exit 1
QG_SC_OLD_TAIL=1 timeout -k 10 60 ./quill-zkvm_amd/micro/sc_capi 20 50 >> gpurun_out/sc_capi_$tag.log 2>&1 || exit 1
timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_$tag.log 2>&1 || exit 1
bash quill-zkvm_amd/micro/sc_ab.sh $tag base=- || exit 1
