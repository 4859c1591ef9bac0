"""HBM traffic per kernel launch and per step from two rocprofv3 PMC passes of a short bench
(scripts/gpu.sh pmc: `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE`, each with --kernel-trace).

FETCH_SIZE is doubled (gfx950 counts 128-B requests at 64 B: MI355X_MICROARCH.md section HBM;
calibrated on librmt's own 8-B/lane pattern in round 1, profiles/r01/hbm_traffic_n4096.md),
WRITE_SIZE is taken as is.  Per step: the dispatches from the second step boundary (a k_dt or
k_dt_part launch: the first kernel of every step) to the end, divided by the steps they cover.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <out.json> [git-rev] [step-start kernels]

(step-start kernels: comma-separated names of the first kernel of a step; default
k_dt,k_dt_part -- config 5's step starts with k_mac_centres_m2)
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = list(csv.DictReader(open(f[0])))
    per = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        did = int(r["Dispatch_Id"])
        name = r["Kernel_Name"].split("(")[0].split("<")[0].strip()
        per[did] = (name, per.get(did, (name, 0.0))[1] + float(r["Counter_Value"]))
    return per


def full(b):
    if not b:
        return {}
    big = [x for x in b if x >= 0.25 * max(b)]
    return {"launches_full": len(big), "bytes_per_full_launch": sum(big) / len(big)}


def main():
    fdir, wdir, out = sys.argv[1:4]
    rev = sys.argv[4] if len(sys.argv) > 4 else ""
    fe = load(fdir, "FETCH_SIZE")
    wr = load(wdir, "WRITE_SIZE")
    kern = defaultdict(lambda: [0, 0.0, 0.0])
    per_launch = defaultdict(list)      # bytes of each dispatch (fetch pass + write pass)
    for did, (name, v) in fe.items():
        k = kern[name]; k[0] += 1; k[1] += 2.0 * v * 1024.0   # FETCH_SIZE is in KiB
    for did, (name, v) in wr.items():
        kern[name][2] += v * 1024.0
    # the two passes are separate runs of the same command: pair the n-th dispatch of a
    # kernel in one with the n-th in the other
    fseq, wseq = defaultdict(list), defaultdict(list)
    for did in sorted(fe):
        fseq[fe[did][0]].append(2.0 * fe[did][1] * 1024.0)
    for did in sorted(wr):
        wseq[wr[did][0]].append(wr[did][1] * 1024.0)
    for n in fseq:
        per_launch[n] = [a + b for a, b in zip(fseq[n], wseq.get(n, []))]
    # per step, from the fetch pass's dispatch order
    order = sorted(fe)
    marks = tuple(sys.argv[5].split(",")) if len(sys.argv) > 5 else ("k_dt", "k_dt_part")
    starts = [d for d in order if fe[d][0] in marks]
    nsteps = len(starts) - 1
    step = {}
    for label, per, scale in (("fetch", fe, 2.0), ("write", wr, 1.0)):
        if len(starts) >= 2:
            # the write pass is a separate run: its dispatch ids are paired by order, so the
            # boundary is the fetch pass's boundary index in sorted order
            ids = sorted(per)
            b = ids[order.index(starts[1])] if len(ids) == len(order) else starts[1]
            tot = sum(v for d, (n, v) in per.items() if d >= b) * scale * 1024.0
            step[label] = tot / nsteps
    res = {"git_rev": rev, "units": "bytes", "fetch_correction": 2.0,
           "kernels": {n: {"launches": c, "fetch_per_launch": f / max(c, 1),
                           "write_per_launch": w / max(c, 1),
                           "bytes_per_launch": (f + w) / max(c, 1),
                           # launches over the whole grid (a kernel also launched on a tile
                           # list, e.g. k_mom_stage's re-run on the extrapolated tiles, moves
                           # a fraction of that): those above a quarter of the largest
                           **full(per_launch[n])}
                       for n, (c, f, w) in sorted(kern.items(), key=lambda kv: -(kv[1][1] + kv[1][2]))},
           "per_step": {"fetch": step.get("fetch"), "write": step.get("write"),
                        "total": (step["fetch"] + step["write"]) if step else None,
                        "steps": nsteps}}
    json.dump(res, open(out, "w"), indent=1)
    print(f"per step: {res['per_step']}")
    for n, k in list(res["kernels"].items())[:12]:
        print(f"{n:40s} x{k['launches']:4d}  {k['bytes_per_launch'] / 1e9:.3f} GB/launch  "
              f"full x{k.get('launches_full', 0)} {k.get('bytes_per_full_launch', 0) / 1e9:.3f}")


if __name__ == "__main__":
    main()
