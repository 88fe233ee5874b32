#!/bin/bash
# Round evidence on the GPU box: full -m gpu suite, the default bench line (the
# driver's command), and the same bench under rocprofv3 --kernel-trace --stats
# (kernel averages per bench leg, from the qg_trace_marker markers, that the
# bench's HIP-event figures must agree with), plus the per-kernel PMC HBM table
# of the bench's probe.  Usage: round_end.sh <tag> [skip-tests]
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r04}
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit 1
fi
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 --detail-out gpurun_out/${tag}_detail.json \
  > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
python3 profiles/pmc_table.py gpurun_out/${tag}_detail.json > gpurun_out/${tag}_pmc_hbm_table.txt
python3 profiles/pmc_table.py gpurun_out/${tag}_detail.json --shapes >> gpurun_out/${tag}_pmc_hbm_table.txt
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run -- \
  python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic \
  --detail-out gpurun_out/${tag}_detail_rocprof.json > gpurun_out/${tag}_bench_under_rocprof.json \
  2> gpurun_out/${tag}_bench_under_rocprof.err || exit 1
python3 profiles/kstats.py gpurun_out/prof_${tag} --legs > gpurun_out/${tag}_kernel_stats_legs.txt
