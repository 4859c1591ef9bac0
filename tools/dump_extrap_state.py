"""Record the extrapolation's input (advected, masked X1, X2 and the pre-advection phi) of
step S of config 4 (soft_disc_in_lid_driven, N=4096, SL), run by the CPU oracle, as raw f64
files for tools/jacobi_sweeps.c.  ANALYSIS INFRASTRUCTURE (imports the oracle; never on the
product path).

    python tools/dump_extrap_state.py [N] [S] [OUTDIR]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
S = int(sys.argv[2]) if len(sys.argv) > 2 else 20
out = sys.argv[3] if len(sys.argv) > 3 else "/tmp/exstate"
os.makedirs(out, exist_ok=True)
O.set_threads(len(os.sched_getaffinity(0)))
O.set_all_cores(True)
seen = {}
orig = O.extrapolate_reference_map


def hook(X1, X2, phi, dx, dy, L):
    seen["args"] = (X1.copy(), X2.copy(), phi.copy())
    return orig(X1, X2, phi, dx, dy, L)


sim = O.SoftDisc(N, "lid")
O_mod = sys.modules[type(sim).__module__]
O_mod.extrapolate_reference_map = hook
for s in range(1, S + 1):
    r = sim.step()
    print(f"step {s} t={r['t']:.6e} cx={r['cx']:.15f}", flush=True)
for name, a in zip(("X1", "X2", "phi"), seen["args"]):
    np.ascontiguousarray(a, dtype=np.float64).tofile(os.path.join(out, f"{name}.bin"))
print("wrote", out)
