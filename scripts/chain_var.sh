#!/bin/bash
# parity of the extrapolation / configs under a chain variant, then A/B bench lines
#   scripts/chain_var.sh OUT VARIANT
set -o pipefail
O=gpurun_out/${1:?out}; V=${2:?variant}
mkdir -p "$O"
RMT_CH_VARIANT=$V timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests -m gpu -k "extrap or configs or step or sim" -s > "$O/tests_v$V.log" 2>&1 \
    || { tail -30 "$O/tests_v$V.log"; exit 1; }
grep -E "passed|failed|^\[config" "$O/tests_v$V.log" | tail -6
bash scripts/ab_env.sh "${1}" "" "RMT_CH_VARIANT=$V" "" "RMT_CH_VARIANT=$V"
