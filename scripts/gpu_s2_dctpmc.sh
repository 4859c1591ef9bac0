#!/bin/bash
set -o pipefail
O=gpurun_out/s2/dctpmc
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/dct_bench.py 4096 5 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -T -f csv -d $O/p1 -o d -- python3 tools/dct_bench.py 4096 2 > $O/p1.log 2>&1 || exit $?
f=$(find $O/p1 -name "*counter_collection.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float)); cnt = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"][:40]; agg[k][r["Counter_Name"]] += float(r["Counter_Value"]); cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    print(k, {c: round(v / cnt[(k, c)]) for c, v in d.items()})
PY
