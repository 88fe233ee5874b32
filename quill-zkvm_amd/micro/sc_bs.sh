#!/bin/bash
# sumcheck big-round block shape A/B on the GPU box (arg: tag): parity digests
# for each variant, bench timings, and the phase trace of each variant
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}_base.log 2>&1 || exit 1
QG_SC_BIG_BS=512 timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}_bs512.log 2>&1 || exit 1
bash quill-zkvm_amd/micro/sc_ab.sh $tag base=- bs512=QG_SC_BIG_BS=512 "bs512b=QG_SC_BIG_BS=512 QG_SC_BIG_BLOCKS=1024" base2=- || exit 1
timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_${tag}_base.log 2>&1 || exit 1
QG_SC_BIG_BS=512 timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_${tag}_bs512.log 2>&1 || exit 1
