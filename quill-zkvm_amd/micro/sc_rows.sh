#!/bin/bash
# batched partial-row loads: sumcheck parity, timing, phase trace
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_generic.py \
  tests/test_gpu_multirank.py tests/test_gpu_hyperplonk.py tests/test_gpu_logup.py -m gpu -x -q \
  -k "sumcheck or zerocheck or generic or hyperplonk or multiset or perm" --timeout 300 \
  --timeout-method thread > gpurun_out/t_rows.log 2>&1 || exit 1
timeout -k 10 200 python3 bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-traffic --no-scaling-modes --steps 20 > gpurun_out/b_rows.log 2>&1 || exit 1
timeout -k 10 200 python3 quill-zkvm_amd/micro/sc_trace.py 20 > gpurun_out/sc_trace_rows.log 2>&1 || exit 1
python3 quill-zkvm_amd/micro/scms.py gpurun_out/b_rows.log
