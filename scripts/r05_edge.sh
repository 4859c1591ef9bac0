#!/bin/bash
# which change fixes the round-4 slab failure with few edge-tile slots.
# The evicting slab test (edge_slots = 8: lists evicted and re-uploaded every step) against
# three builds: nodrain_copy = no drain, plain hipMemcpy upload (round 4's failing code);
# drain_copy = round 4's drain, plain upload; default = stream-ordered upload (+ drain).
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"
for v in nodrain_copy drain_copy default; do
    L=pyrmt_amd/librmt_$v.so; [ $v = default ] && L=pyrmt_amd/librmt.so
    RMT_LIB=$L timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread \
        tests/test_distributed.py -k "evicting or test_config4_slab_step_N4096" > "$O/$v.log" 2>&1
    echo "$v rc=$? $(tail -1 $O/$v.log)"
done
