#!/bin/bash
# sumcheck timing A/B on the GPU box: arg 1 = tag, then NAME=ENV pairs ("-" = defaults)
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%=*}; envs=${spec#*=}
  [ "$envs" = "-" ] && envs=""
  env $envs timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 \
    --no-cpu-baseline --no-traffic --no-scaling-modes --no-host-input --steps 20 --detail-out '' \
    > gpurun_out/b_sc_${tag}_$name.log 2>&1 || exit 1
done
