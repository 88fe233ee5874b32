#!/bin/bash
# HyperPlonk (2^20 rows) + headline MSM under alternating environment settings.
# Usage: micro/hp_env_ab2.sh <out> <env-setting or -> ...   ("-" = defaults)
out=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    echo "== $v"
    e=(); [ "$v" != "-" ] && e=($v)
    env "${e[@]}" timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-traffic \
      --no-cpu-baseline --no-scaling-modes --no-sumcheck --log-mle 0 --log-logup 0 \
      --log-msm-small 0 --no-host-input --detail-out "" 2>/dev/null | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
k = d['kernels_ms']; h = d.get('hyperplonk', {}); p = h.get('parts_ms_rank0', {})
print('msm2p24', d['ms_per_step'], 'acc', k['msm_accumulate']['ms_avg'], 'red', k['msm_reduce']['ms_avg'],
      'ok', d['commitment_verified'], '| hp', h.get('ms'),
      {x: round(p.get(x, 0), 1) for x in ('msm_accumulate', 'msm_reduce', 'msm_bucketing_side', 's_polynomial')})
" || exit 1
  done
done > "$out" 2>&1
cat "$out"
