"""Config-4 oracle fixture at the bench's length (TEST INFRASTRUCTURE): soft_disc_in_lid_driven
at N=4096 for 100 steps (the loop of soft_disc_in_lid_driven.py:206-235, restated by
oracle.SoftDisc, pinned bit-exact to the reference's fixtures by tests/test_oracle_golden.py).

~8 s per oracle step here (all-cores mode: same bits), too long inside a GPU test, so the run
is summarised once into a small fixture: per-step (t, dt, cx, cy, minJ, maxJ), SHA-256 digests
of the final maps, strided samples of the final X1, X2, u, v, p, and the full row / column
through the disc centre.

Usage:  python tests/golden/gen_config4_100.py   (writes tests/golden/lid4096_100_oracle.npz)
"""
import hashlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import oracle as O          # noqa: E402

N, STEPS, STRIDE = 4096, 100, 32


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def main():
    O.set_threads(len(os.sched_getaffinity(0)))
    O.set_all_cores(True)
    sim = O.SoftDisc(N, "lid")
    t0 = time.time()
    diag = []
    for s in range(1, STEPS + 1):
        r = sim.step()
        diag.append([r["t"], r["dt"], r["cx"], r["cy"], r["minJ"], r["maxJ"]])
        if s % 10 == 0:
            print(f"step {s}/{STEPS} {time.time() - t0:.0f} s", flush=True)
    jc, ic = int(0.5 * (N - 1)), int(0.6 * (N - 1))
    out = {"N": np.array(N), "steps": np.array(STEPS), "stride": np.array(STRIDE),
           "diag": np.array(diag), "rowcol": np.array([jc, ic])}
    for name, f in (("X1", sim.X1), ("X2", sim.X2), ("u", sim.a), ("v", sim.b), ("p", sim.p),
                    ("phi", sim.phi)):
        out[f"{name}_sha"] = np.array(digest(f))
        out[f"{name}_sub"] = f[::STRIDE, ::STRIDE].copy()
        out[f"{name}_row"] = f[jc].copy()
        out[f"{name}_col"] = f[:, ic].copy()
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lid4096_100_oracle.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path)} B) in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
