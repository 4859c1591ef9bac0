"""Dump the extrapolation inputs of the config-4 loop (oracle.SoftDisc, the reference's
arithmetic) at chosen steps, for the CPU model of the chain's event fold
(tools/chain_events.c).  Per dumped step k: the masked advected map (X1, X2) the
extrapolation reads, the pre-advection level set phi, the previous step's map (the chain's
prediction source, sim.hip's ex_pred) and the extrapolated map (the reference's answer).

    python tools/dump_ex_state.py N STEPS OUTDIR [k1,k2,...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    N, steps, out = int(sys.argv[1]), int(sys.argv[2]), sys.argv[3]
    want = {int(s) for s in sys.argv[4].split(",")} if len(sys.argv) > 4 else {steps}
    os.makedirs(out, exist_ok=True)
    from oracle import oracle as O
    O.set_threads(len(os.sched_getaffinity(0)))
    O.set_all_cores(True)
    sim = O.SoftDisc(N, "lid")
    orig = O.extrapolate_reference_map
    state = {"k": 0}

    def hooked(X1, X2, phi, dx, dy, layers):
        r1, r2 = orig(X1, X2, phi, dx, dy, layers)
        if state["k"] in want:
            k = state["k"]
            for name, a in (("X1", X1), ("X2", X2), ("phi", phi), ("P1", sim.X1),
                            ("P2", sim.X2), ("E1", r1), ("E2", r2)):
                np.save(os.path.join(out, f"k{k:03d}_{name}.npy"), np.ascontiguousarray(a))
            with open(os.path.join(out, f"k{k:03d}_meta.txt"), "w") as f:
                f.write(f"{N} {float(dx)!r} {float(dy)!r} {layers}\n")
            print(f"dumped step {k}", flush=True)
        return r1, r2

    O.extrapolate_reference_map = hooked
    t0 = time.time()
    for k in range(1, steps + 1):
        state["k"] = k
        sim.step()
        print(f"step {k}/{steps} {time.time() - t0:.0f} s", flush=True)


if __name__ == "__main__":
    main()
