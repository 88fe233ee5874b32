#!/bin/bash
# sumcheck big-round scheduling A/B on the GPU box (arg: tag): per-wave traces
# (static 256 / 512-thread blocks, dynamic wave chunks), parity digests, timings
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
for v in "base=" "bs512=QG_SC_BIG_BS=512" "dyn=QG_SC_DYN=1"; do
  name=${v%%=*}; envs=${v#*=}
  env $envs timeout -k 10 120 python quill-zkvm_amd/micro/sc_wtrace.py 20 > gpurun_out/wtrace_${tag}_$name.log 2>&1 || exit 1
  env $envs timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_${tag}_$name.log 2>&1 || exit 1
  env $envs timeout -k 10 120 python quill-zkvm_amd/micro/sc_ab.py 20 > gpurun_out/sc_dig_${tag}_$name.log 2>&1 || exit 1
done
bash quill-zkvm_amd/micro/sc_ab.sh $tag base=- dyn=QG_SC_DYN=1 "dyn512=QG_SC_DYN=1 QG_SC_BIG_BS=512" "dyn3=QG_SC_DYN=1 QG_SC_BIG_BLOCKS=768" base2=- dyn2=QG_SC_DYN=1 || exit 1
