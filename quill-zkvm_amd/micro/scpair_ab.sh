#!/bin/bash
# paired-multiply sumcheck A/B: sumcheck parity with the paired build, then the
# bench's sumcheck leg alternating between the two builds (swapped in place on
# the box's copy of the tree)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py tests/test_gpu_hyperplonk.py \
  -m gpu -x -q -k "sumcheck or zerocheck or hyperplonk" --timeout 200 \
  --timeout-method thread > gpurun_out/t_scpair.log 2>&1 || exit 1
for r in 1 2; do
  for v in scold scnew; do
    cp quill-zkvm_amd/micro/lib_$v.so quill-zkvm_amd/libquill_gpu.so
    timeout -k 10 200 python bench.py --log-msm 16 --log-mle 0 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
      --no-traffic --no-scaling-modes --steps 20 > gpurun_out/b_${v}_$r.json 2> gpurun_out/b_${v}_$r.err || exit 1
  done
done
