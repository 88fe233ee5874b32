#!/bin/bash
# host-input commit pipelining check (arg: tag): parity, then the bench's
# msm_host_input leg for several piece counts
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "msm or kzg or commit" \
  --timeout 200 --timeout-method thread > gpurun_out/t_host_$tag.log 2>&1 || exit 1
for p in 1 2 4 8; do
  QG_MSM_PIECES=$p timeout -k 10 300 python -u bench.py --no-sumcheck --log-mle 0 --log-logup 0 --log-hp-rows 0 \
    --no-cpu-baseline --no-traffic --no-scaling-modes --steps 5 --detail-out gpurun_out/host_${tag}_p$p.json \
    > gpurun_out/host_${tag}_p$p.out 2>&1 || exit 1
done
