#!/bin/bash
# two-pairs-per-step sumcheck A/B on the GPU box (arg: tag)
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}_base.log 2>&1 || exit 1
QG_SC_TWO=1 timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}_two.log 2>&1 || exit 1
QG_SC_TWO=1 timeout -k 10 120 python quill-zkvm_amd/micro/sc_wtrace.py 20 > gpurun_out/wtrace_${tag}_two.log 2>&1 || exit 1
QG_SC_TWO=1 timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_${tag}_two.log 2>&1 || exit 1
bash quill-zkvm_amd/micro/sc_ab.sh $tag base=- two=QG_SC_TWO=1 base2=- two2=QG_SC_TWO=1 || exit 1
