#!/bin/bash
# sumcheck check + timing + phase trace on the GPU box (arg: tag)
#   gpurun -- 'bash quill-zkvm_amd/micro/sc_check.sh <tag>'
# needs libquill_gpu.so and micro/libquill_gpu_trace.so built beforehand (make; make trace)
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py \
  tests/test_gpu_hyperplonk.py tests/test_gpu_multirank.py tests/test_gpu_generic.py -m gpu -x -q \
  -k "sumcheck or zerocheck or hyperplonk or generic" --timeout 200 \
  --timeout-method thread > gpurun_out/t_sc_$tag.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-traffic --no-scaling-modes --steps 20 --detail-out '' > gpurun_out/b_sc_$tag.log 2>&1 || exit 1
timeout -k 10 120 python quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_$tag.log 2>&1 || exit 1
# A/B: every point evaluated in every big round; 768 big-round blocks (3 waves / SIMD)
QG_SC_NO_SKIP0=1 timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 \
  --no-cpu-baseline --no-traffic --no-scaling-modes --steps 20 --detail-out '' > gpurun_out/b_sc_${tag}_noskip.log 2>&1 || exit 1
QG_SC_BIG_BLOCKS=768 timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 \
  --no-cpu-baseline --no-traffic --no-scaling-modes --steps 20 --detail-out '' > gpurun_out/b_sc_${tag}_768.log 2>&1 || exit 1
QG_SC_BIG_BLOCKS=1024 timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 \
  --no-cpu-baseline --no-traffic --no-scaling-modes --steps 20 --detail-out '' > gpurun_out/b_sc_${tag}_1024.log 2>&1 || exit 1
