#!/bin/bash
# Config-5 A/B of two library builds: the MAC GPU tests on B, then interleaved config-5 bench
# lines.   scripts/r05_cfg5ab.sh OUT LIB_A LIB_B [extra env for B]
set -o pipefail
O=gpurun_out/${1:?out}; A=${2:?lib a}; B=${3:?lib b}
mkdir -p "$O"; export TMPDIR=/tmp
RMT_LIB=$B timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_mac.py tests/test_gpu_configs.py -k "mac or config5" > "$O/tests.log" 2>&1 \
    || { tail -30 "$O/tests.log"; exit 1; }
tail -2 "$O/tests.log"
for L in "$A" "$B"; do
    RMT_LIB=$L timeout -k 10 200 python -u tools/mac_sha.py 8192 3 > "$O/sha_$(basename "$L" .so).txt" 2>&1 \
        || { tail -5 "$O/sha_$(basename "$L" .so).txt"; exit 1; }
    tail -1 "$O/sha_$(basename "$L" .so).txt"
done
k=0
for L in "$A" "$B" "$A" "$B"; do
    k=$((k + 1)); t=$(basename "$L" .so)
    RMT_LIB=$L timeout -k 10 300 python -u bench.py --config 5 --no-cpu-baseline --steps 20 > "$O/b_${k}_$t.log" 2>&1 \
        || { tail -20 "$O/b_${k}_$t.log"; exit 1; }
    echo "$t $(tail -1 "$O/b_${k}_$t.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['ms_per_step'],3))")"
done
