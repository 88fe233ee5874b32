#!/bin/bash
# Logup column check (arg: tag): parity tests, the bench's logup leg, kernel trace
set -o pipefail
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "logup or lookup or multiset or permutation or set_inclusion or hyperplonk or bingcd" \
  --timeout 200 --timeout-method thread > gpurun_out/t_lg_$tag.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --log-msm 16 --no-sumcheck --log-mle 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-scaling-modes --steps 10 --detail-out gpurun_out/lg_${tag}.json > gpurun_out/lg_${tag}.out 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lg_$tag -o run -- \
  python3 -u bench.py --log-msm 16 --no-sumcheck --log-mle 0 --log-hp-rows 0 --no-cpu-baseline --no-traffic \
  --no-scaling-modes --steps 10 --detail-out '' > gpurun_out/lg_${tag}_prof.out 2>&1 || exit 1
python3 profiles/kstats.py gpurun_out/lg_$tag logup > gpurun_out/lg_$tag.txt || exit 1
QG_LOGUP_FUSED=1 timeout -k 10 300 python -u bench.py --log-msm 16 --no-sumcheck --log-mle 0 --log-hp-rows 0 --no-cpu-baseline \
  --no-scaling-modes --steps 10 --detail-out gpurun_out/lg_${tag}_1p.json > gpurun_out/lg_${tag}_1p.out 2>&1 || exit 1
