#!/bin/bash
# A/B of the MSM chunk rule (QG_MSM_EQSPLIT=k: equal chunks over k rounds of the
# resident waves; 0 = the power-of-two rule), alternating, headline 2^24 and
# the HyperPlonk leg.  Usage: micro/msm_eqsplit_ab.sh <out> <values...>
out=$1; shift
for rep in 1 2; do
  for v in "$@"; do
    echo "== QG_MSM_EQSPLIT=$v"
    QG_MSM_EQSPLIT=$v timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-traffic \
      --no-cpu-baseline --no-scaling-modes --no-sumcheck --log-mle 0 --log-logup 0 \
      --log-msm-small 0 --no-host-input --detail-out "" 2>/dev/null | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
k = d['kernels_ms']; h = d.get('hyperplonk', {}); p = h.get('parts_ms_rank0', {})
print('msm2p24', d['ms_per_step'], 'acc', k['msm_accumulate']['ms_avg'], 'red', k['msm_reduce']['ms_avg'],
      'buck', k['msm_bucketing']['ms_avg'], 'ok', d['commitment_verified'],
      '| hp', h.get('ms'), 'acc', round(p.get('msm_accumulate', 0), 1), 'red', round(p.get('msm_reduce', 0), 1))
" || exit 1
  done
done > "$out" 2>&1
cat "$out"
