#!/bin/bash
# sumcheck C-ABI timing under env settings, alternating: sc_env_ab.sh <nv> <steps> <rounds> NAME=ENV...
# ("-" = defaults), e.g. base=- pl16=QG_SC_PERS_LOG=16
set -o pipefail
cd "$(dirname "$0")/.."
nv=$1; steps=$2; rounds=$3; shift 3
for i in $(seq "$rounds"); do
  for spec in "$@"; do
    name=${spec%%=*}; envs=${spec#*=}
    [ "$envs" = "-" ] && envs=""
    printf '%s ' "$name"
    env $envs timeout -k 5 60 micro/sc_capi "$nv" "$steps" || exit 1
  done
done
