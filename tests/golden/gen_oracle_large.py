"""Large-size oracle fixtures (TEST INFRASTRUCTURE): config 5, mac_multi_disc_lid at N=8192.

The oracle (oracle/mac_oracle.py, pinned bit-exact to the reference's own fixtures by
tests/test_oracle_golden.py) needs ~90 s per step at N=8192 (NumPy on 512 MiB planes), too
long to run inside a GPU test, so its first two steps are run here once and summarised into
a small fixture: the per-step diagnostics, SHA-256 digests of every disc's (X1, X2, phi)
after each step (bit-exact comparisons), strided samples of u, v, p and of the maps, and the
full rows / columns through each disc centre (tolerance comparisons).

Usage:  python tests/golden/gen_oracle_large.py   (writes tests/golden/mac8192_oracle.npz)
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O          # noqa: E402
from oracle import mac_oracle as M      # noqa: E402

N, STEPS, STRIDE = 8192, 2, 64


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def summarise(sim, out, s):
    out[f"u_s{s}"] = sim.u[::STRIDE, ::STRIDE].copy()
    out[f"v_s{s}"] = sim.v[::STRIDE, ::STRIDE].copy()
    out[f"p_s{s}"] = sim.p[::STRIDE, ::STRIDE].copy()
    for k, (R, cx, cy) in enumerate(sim.specs):
        X1, X2 = sim.refs[k]
        phi = sim.phis[k]
        jc, ic = int(cy * N), int(cx * N)
        for name, f in (("X1", X1), ("X2", X2), ("phi", phi)):
            out[f"{name}_d{k}_s{s}_sha"] = np.array(digest(f))
            out[f"{name}_d{k}_s{s}_row"] = f[jc].copy()
            out[f"{name}_d{k}_s{s}_col"] = f[:, ic].copy()
            out[f"{name}_d{k}_s{s}_sub"] = f[::STRIDE, ::STRIDE].copy()
        out[f"rowcol_d{k}"] = np.array([jc, ic])


def main():
    O.set_threads(os.cpu_count() or 1)
    O.set_all_cores(True)       # same results bit for bit; only faster
    t0 = time.time()
    sim = M.MacMultiDisc(N)
    out = {"N": np.array(N), "stride": np.array(STRIDE), "specs": np.array(sim.specs),
           "dt": np.array(sim.dt)}
    print(f"init {time.time() - t0:.1f} s", flush=True)
    diag = []
    for s in range(1, STEPS + 1):
        t1 = time.time()
        r = sim.step()
        diag.append([r["t"], r["dt"], r["minJ"], r["maxJ"], *r["cx"], *r["cy"]])
        summarise(sim, out, s)
        print(f"step {s}: {time.time() - t1:.1f} s  {r}", flush=True)
    out["diag"] = np.array(diag, dtype=np.float64)
    path = os.path.join(ROOT, "tests", "golden", "mac8192_oracle.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
