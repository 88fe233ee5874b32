#!/bin/bash
# paired-butterfly NTT A/B: S-polynomial / ML-open parity with the new build,
# then the bench's ML-open leg alternating the two builds (swapped in place on
# the box's copy of the tree)
set -o pipefail
export TMPDIR=/tmp
cp quill-zkvm_amd/micro/lib_nttnew.so quill-zkvm_amd/libquill_gpu.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -m gpu -x -q \
  -k "spoly or s_poly or ntt or mle or open" --timeout 250 --timeout-method thread > gpurun_out/t_ntt.log 2>&1 || exit 1
for r in 1 2; do
  for v in ntthead nttnew; do
    cp quill-zkvm_amd/micro/lib_$v.so quill-zkvm_amd/libquill_gpu.so
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/nt_${v}_$r -o run -- python3 bench.py --log-msm 16 --log-logup 0 --log-hp-rows 0 --no-cpu-baseline \
      --no-traffic --no-scaling-modes --steps 3 > gpurun_out/nt_${v}_$r.json 2> gpurun_out/nt_${v}_$r.err || exit 1
    python3 profiles/kstats.py gpurun_out/nt_${v}_$r > gpurun_out/nt_${v}_$r.txt || exit 1
  done
done
