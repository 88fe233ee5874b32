#!/bin/bash
# SQ counters of the sumcheck kernels (two-lane and QG_SC_V1), one pass each
set -o pipefail
export TMPDIR=/tmp
P="--log-msm 16 --log-sumcheck 20 --log-logup 0 --log-mle 0"
C1="SQ_WAVES,SQ_INSTS_VALU,SQ_INSTS_VMEM_RD,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_INSTS_SALU,SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
timeout -k 10 120 python3 pmc_traffic.py $C1 -- $P > gpurun_out/sc_pmc_two.json 2> gpurun_out/sc_pmc_two.err || exit 1
QG_SC_V1=1 timeout -k 10 120 python3 pmc_traffic.py $C1 -- $P > gpurun_out/sc_pmc_v1.json 2> gpurun_out/sc_pmc_v1.err || exit 1
