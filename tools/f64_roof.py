"""fp64 VALU roof of k_mom_stage from scripts/pmc_f64.sh: the measured FMA peak
(tools/ubench_f64) and one SQ counter pass over the kernel's launches.

Per full-grid launch: FLOP = 64 lanes x (ADD + MUL + TRANS + 2 FMA) F64 wave-instructions
(exec masks ignored: an upper bound on useful flops), and the VALU issue floor: gfx950 issues
a wave64 f64 instruction in 4 cycles and any other VALU instruction in 2 (MI355X_MICROARCH.md
row 'vector-instruction ISSUE cost'; 4 for f64 at the measured FMA rate), over 1024 SIMDs at
the clock the FMA probe implies.

    python tools/f64_roof.py gpurun_out/<out> profiles/r02/f64_roof_n4096.json [git-rev]
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

out_dir, dst = sys.argv[1], sys.argv[2]
rev = sys.argv[3] if len(sys.argv) > 3 else None
m = re.search(r"(\d+) CUs, ([\d.]+) ms, ([\d.]+) TFLOP/s", open(os.path.join(out_dir, "ubench_f64.log")).read())
cus, peak = int(m.group(1)), float(m.group(3))
simds = 4 * cus
clock = peak * 1e12 / (simds * 16 * 2)          # 16 f64 FMA lanes per SIMD per cycle
f = glob.glob(os.path.join(out_dir, "f64", "*counter_collection.csv"))[0]
per = defaultdict(lambda: defaultdict(float))
for r in csv.DictReader(open(f)):
    per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
full = [c for c in per.values() if c["SQ_INSTS_VALU"] >= 0.25 * max(x["SQ_INSTS_VALU"] for x in per.values())]
avg = {k: sum(c[k] for c in full) / len(full) for k in full[0]}
f64 = avg["SQ_INSTS_VALU_ADD_F64"] + avg["SQ_INSTS_VALU_MUL_F64"] + avg["SQ_INSTS_VALU_FMA_F64"] + avg["SQ_INSTS_VALU_TRANS_F64"]
flop = 64 * (f64 + avg["SQ_INSTS_VALU_FMA_F64"])
issue_cycles = (4 * f64 + 2 * (avg["SQ_INSTS_VALU"] - f64)) / simds
res = {"git_rev": rev, "kernel": "k_mom_stage", "launches_full": len(full),
       "valu_wave_insts_per_launch": avg["SQ_INSTS_VALU"], "f64_wave_insts_per_launch": f64,
       "counters_per_launch": avg, "flop_per_launch": flop,
       "fma_peak_tflops_measured": peak, "clock_ghz_implied": clock / 1e9,
       "valu_issue_floor_ms": issue_cycles / clock * 1e3,
       "source": "scripts/pmc_f64.sh (tools/ubench_f64 + rocprofv3 --pmc SQ_INSTS_VALU_*_F64)"}
json.dump(res, open(dst, "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "counters_per_launch"}, indent=1))
