#!/bin/bash
# sumcheck 2^20 timing over big-round block counts (QG_SC_BIG_BLOCKS)
set -o pipefail
B="python3 bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline --no-traffic --no-scaling-modes --steps 20"
for nb in 512 640 768 1024; do
  QG_SC_BIG_BLOCKS=$nb timeout -k 10 200 $B > gpurun_out/b_scb_$nb.log 2>&1 || exit 1
done
