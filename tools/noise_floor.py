"""Reference noise floor of the loop, measured
with the oracle (the C restatement of the reference, bit-exact against its fixtures):

  mode 0  the reference's extrapolation arithmetic
  mode 1  every extrapolation weight nudged +1 ulp (the App. A.5 experiment)
  mode 2  the centred restatement of each fit that librmt's parallel extrapolation computes

Each case runs the driver loop (oracle.SoftDisc) from the driver's initial state for the
given steps in every mode and reports, per step, the largest deviation of modes 1 and 2
from mode 0 in the centroid, J min / max and (Taylor-Green) the energies; plus the largest
band-value deviation of the map.  One process per mode (fork), oracle in all-cores mode.

  python tools/noise_floor.py CASE N STEPS OUT.json     CASE in {lid, tg}
"""
import json
import os
import sys
import time
from multiprocessing import get_context

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(args):
    case, N, steps, mode, threads = args
    from oracle import oracle as O
    O.set_threads(threads)
    O.set_all_cores(True)
    O.set_ex_mode(mode)
    sim = O.SoftDisc(N, case, "semilagrangian" if case == "lid" else "weno5")
    recs = []
    t0 = time.time()
    for k in range(steps):
        recs.append(sim.step(energies=(case == "tg")))
        if k % 5 == 0:
            print(f"[mode {mode}] step {k + 1}/{steps} {time.time() - t0:.0f} s", flush=True)
    keys = [k for k in recs[0] if isinstance(recs[0][k], float)]
    return mode, {k: [r[k] for r in recs] for k in keys}, sim.X1, sim.X2, sim.a, sim.p


def main():
    case, N, steps, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    ncpu = len(os.sched_getaffinity(0))
    th = max(1, ncpu // 3)
    with get_context("fork").Pool(3) as pool:
        res = pool.map(run, [(case, N, steps, m, th) for m in (0, 1, 2)])
    res = {r[0]: r for r in res}
    base = res[0][1]
    summ = {"case": case, "N": N, "steps": steps, "modes": {}}
    for m in (1, 2):
        rec = res[m][1]
        d = {}
        for k in base:
            a, b = np.array(base[k]), np.array(rec[k])
            absd = np.abs(a - b)
            rel = absd / np.maximum(np.abs(a), 1e-300)
            d[k] = {"max_abs": float(absd.max()), "max_rel": float(rel.max()),
                    "final_abs": float(absd[-1]), "per_step_rel": [float(x) for x in rel]}
        for name, idx in (("X1", 2), ("X2", 3), ("u", 4), ("p", 5)):
            d["field_" + name + "_max_abs"] = float(np.abs(res[0][idx] - res[m][idx]).max())
        summ["modes"][{1: "nudge_1ulp", 2: "centred"}[m]] = d
    json.dump(summ, open(out, "w"), indent=1)
    for m, d in summ["modes"].items():
        print(m, {k: (v["max_rel"] if isinstance(v, dict) else v) for k, v in d.items()})


if __name__ == "__main__":
    main()
