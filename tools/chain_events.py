"""Run the CPU model of the chain's event fold (tools/chain_events.c) on a dumped config-4
extrapolation state (tools/dump_ex_state.py) and report how often the event walk would
fall back to the exact fold, how many events a fit needs, and that every accepted event
result equals the exact fold bit for bit.

    python tools/chain_events.py DUMPDIR k [pred_mode]    (pred_mode 1: predict 0.0)
"""
import ctypes
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = "/tmp/chain_events.so"


def main():
    d, k = sys.argv[1], int(sys.argv[2])
    pm = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC",
                    os.path.join(HERE, "chain_events.c"), "-o", SO, "-lm"], check=True)
    lib = ctypes.CDLL(SO)
    P = ctypes.c_void_p
    lib.ce_run.restype = ctypes.c_long
    lib.ce_run.argtypes = [P, P, P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                           ctypes.c_double, ctypes.c_int, P, P, P, ctypes.c_int]
    ld = lambda n: np.load(os.path.join(d, f"k{k:03d}_{n}.npy"))
    X1, X2, phi, P1, P2, E1, E2 = (ld(n) for n in ("X1", "X2", "phi", "P1", "P2", "E1", "E2"))
    N, dx, dy, layers = open(os.path.join(d, f"k{k:03d}_meta.txt")).read().split()
    num = lambda s: float(s.replace("np.float64(", "").rstrip(")"))
    N, dx, dy, layers = int(N), num(dx), num(dy), int(layers)
    o1, o2 = np.empty_like(X1), np.empty_like(X2)
    st = np.zeros(1024, dtype=np.int64)
    p = lambda a: a.ctypes.data_as(P)
    filled = lib.ce_run(p(X1), p(X2), p(phi), p(P1), p(P2), N, N, dx, dy, layers, p(o1), p(o2),
                        p(st), pm)
    same = np.array_equal(o1.view(np.int64), E1.view(np.int64)) and \
        np.array_equal(o2.view(np.int64), E2.view(np.int64))
    fits, fdyn, fb, mm, fbb, fbm, fbp = st[:7]
    worst = st[7:8].view(np.float64)[0]
    print(f"step {k}: filled {filled}, output == reference: {same}")
    print(f"fits {fits} (with dynamic terms {fdyn}); fallback {fb} ({100 * fb / max(fits, 1):.3f} %:"
          f" binade {fbb}, margin {fbm}, path {fbp}); MISMATCHES {mm}; worst |d|/M {worst:.3g}")

    def hist(name, h):
        h = np.asarray(h)
        tot = h.sum()
        nz = np.nonzero(h)[0]
        cum = np.cumsum(h) / max(tot, 1)
        mean = (np.arange(len(h)) * h).sum() / max(tot, 1)
        q = {pp: int(np.searchsorted(cum, pp)) for pp in (0.5, 0.9, 0.99)}
        print(f"{name}: mean {mean:.2f} median {q[0.5]} p90 {q[0.9]} p99 {q[0.99]} max {nz.max() if len(nz) else 0}")

    hist("events per lane (max over the 6 sums)", st[8:72])
    hist("events from the critical term on", st[72:136])
    hist("dynamic terms per fit", st[136:232])
    hist("static events after the critical term", st[232:296])
    print(f"union: fallback {st[488]} mismatches {st[489]}")
    hist("union events per fit", st[296:392])
    hist("union events from the critical term on", st[392:488])
    print(f"delta trick: fallback {st[682]} mismatches {st[683]}")
    hist("real events from the critical term on", st[490:586])
    hist("dependent ops after the arrival", st[586:682])


if __name__ == "__main__":
    main()
