"""Per-kernel summary of scripts/r05_prof.sh's counter passes: mean duration (from the
kernel trace of the counter runs), HBM bytes (FETCH_SIZE x 2 on gfx950, WRITE_SIZE as is:
MI355X_MICROARCH.md section HBM), achieved GB/s, VALU wave-instructions and the VALU-busy
and wait shares of the wave cycles.   python tools/pmc_summary.py OUT_DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]


def counters(sub):
    f = glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}, {}
    per = defaultdict(lambda: defaultdict(float))
    name = {}
    for r in csv.DictReader(open(f[0])):
        d = int(r["Dispatch_Id"])
        name[d] = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    return per, name


def durations(sub):
    f = glob.glob(os.path.join(out, sub, "**", "*kernel_trace.csv"), recursive=True)
    dur = {}
    for r in csv.DictReader(open(f[0])) if f else []:
        dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    return dur


agg = defaultdict(lambda: defaultdict(list))
for sub in ("pa", "pf", "pw"):
    per, name = counters(sub)
    dur = durations(sub)
    for d, cs in per.items():
        k = name[d]
        for c, v in cs.items():
            agg[k][c].append(v)
        if d in dur and sub == "pa":
            agg[k]["dur"].append(dur[d])


def mean(x):
    return sum(x) / len(x) if x else float("nan")


rows = []
for k, cs in agg.items():
    t = mean(cs["dur"])
    fetch = 2 * mean(cs.get("FETCH_SIZE", [])) * 1024   # FETCH_SIZE / WRITE_SIZE are in KB
    write = mean(cs.get("WRITE_SIZE", [])) * 1024
    wc = mean(cs.get("SQ_WAVE_CYCLES", []))
    rows.append((t * len(cs["dur"]), k, len(cs["dur"]), t, fetch, write,
                 mean(cs.get("SQ_INSTS_VALU", [])), mean(cs.get("SQ_ACTIVE_INST_VALU", [])) / wc if wc else 0,
                 mean(cs.get("SQ_WAIT_ANY", [])) / wc if wc else 0,
                 mean(cs.get("SQ_WAIT_INST_ANY", [])) / wc if wc else 0,
                 mean(cs.get("SQ_INSTS_LDS", [])), mean(cs.get("SQ_INSTS_SALU", []))))
rows.sort(reverse=True)
print(f"{'kernel':28s} {'n':>4s} {'us':>8s} {'fetch MB':>9s} {'write MB':>9s} {'GB/s':>7s} "
      f"{'VALU Mi':>8s} {'valu%':>6s} {'wait%':>6s} {'wins%':>6s} {'LDS Mi':>7s} {'SALU Mi':>7s}")
for tot, k, n, t, f, w, valu, vb, wa, wi, lds, salu in rows:
    print(f"{k[:28]:28s} {n:4d} {t * 1e6:8.1f} {f / 1e6:9.1f} {w / 1e6:9.1f} "
          f"{(f + w) / t / 1e9 if t else 0:7.0f} {valu / 1e6:8.2f} {100 * vb:6.1f} {100 * wa:6.1f} "
          f"{100 * wi:6.1f} {lds / 1e6:7.2f} {salu / 1e6:7.2f}")
