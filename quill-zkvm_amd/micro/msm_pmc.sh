#!/bin/bash
# SQ counters of the MSM kernels at 2^24 (one rocprofv3 pass per group); arg: tag
set -o pipefail
export TMPDIR=/tmp
tag=$1
P="--log-msm 24 --no-sumcheck --log-logup 0 --log-mle 0"
G1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU"
G2="SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_ACTIVE_INST_ANY,SQ_INST_CYCLES_VMEM_RD,SQ_INSTS_VMEM_WR,SQ_ACTIVE_INST_SCA,SQ_INSTS_SMEM,SQ_WAIT_INST_LDS"
k=0
for G in $G1 $G2; do
  k=$((k+1))
  timeout -k 10 150 python3 pmc_traffic.py $G -- $P > gpurun_out/msm_pmc_${tag}_$k.json 2> gpurun_out/msm_pmc_${tag}_$k.err || exit 1
done
