#!/bin/bash
# Round-end evidence on the GPU box: full -m gpu suite, the default bench line,
# and the same bench under rocprofv3 --kernel-trace --stats (kernel averages
# that the bench's HIP-event figures must agree with).  Usage: round_end.sh <tag>
set -o pipefail
export TMPDIR=/tmp
tag=${1:-r02}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_gpu_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || exit 1
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag} -o run -- \
  python3 -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/${tag}_bench_under_rocprof.json \
  2> gpurun_out/${tag}_bench_under_rocprof.err || exit 1
python3 profiles/kstats.py gpurun_out/prof_${tag} > gpurun_out/${tag}_kernel_stats.txt
