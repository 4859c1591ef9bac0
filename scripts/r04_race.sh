#!/bin/bash
# repeat one GPU test under two libraries (diagnosis of a schedule-dependent mismatch)
#   scripts/r04_race.sh OUT TEST_EXPR LIB1 LIB2 [reps]
set -o pipefail
O=gpurun_out/${1:?out}; mkdir -p "$O"; shift
T=$1; shift; L1=$1; shift; L2=$1; shift; R=${1:-2}
for L in "$L1" "$L2"; do for r in $(seq 1 $R); do
  RMT_LIB=$L timeout -k 10 300 python -u -m pytest -q -x --timeout 280 --timeout-method thread tests -m gpu -k "$T" > "$O/$(basename $L)_$r.log" 2>&1
  echo "$L rep $r rc=$? $(tail -1 $O/$(basename $L)_$r.log)"
done; done
