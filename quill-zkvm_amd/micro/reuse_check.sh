#!/bin/bash
# transform reuse: parity (ML-open + HyperPlonk) then the HyperPlonk bench leg
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_hyperplonk.py tests/test_gpu_verifier.py \
  tests/test_gpu_headline.py -m gpu -x -q -k "mle or hyperplonk or microbench or verif" --timeout 300 \
  --timeout-method thread > gpurun_out/t_reuse.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --log-msm 16 --log-logup 0 --no-cpu-baseline --no-traffic \
  --no-scaling-modes > gpurun_out/b_reuse.json 2> gpurun_out/b_reuse.err || exit 1
