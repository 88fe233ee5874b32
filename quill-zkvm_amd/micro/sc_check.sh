#!/bin/bash
# sumcheck check + timing + phase trace on the GPU box (arg: tag)
set -o pipefail
export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_hyperplonk.py \
  tests/test_gpu_multirank.py -m gpu -x -q -k "sumcheck or zerocheck or hyperplonk" --timeout 200 \
  --timeout-method thread > gpurun_out/t_sc_$tag.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-traffic --steps 20 > gpurun_out/b_sc_$tag.log 2>&1 || exit 1
timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_$tag.log 2>&1
QG_SC_PF=1 timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-traffic --steps 20 > gpurun_out/b_sc_${tag}_pf.log 2>&1
