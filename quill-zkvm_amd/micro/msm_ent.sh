#!/bin/bash
# accumulate with 16-B entry loads: MSM parity, then the bench headline with PMC traffic
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q \
  -k "msm or kzg or commit" --timeout 200 --timeout-method thread > gpurun_out/t_ent.log 2>&1 || exit 1
timeout -k 10 800 python -u bench.py --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-scaling-modes > gpurun_out/b_ent.json 2> gpurun_out/b_ent.err || exit 1
