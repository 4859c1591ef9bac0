"""Prototype of the parallel extrapolation (segment-affine solve), host-side numpy/Python,
for the design numbers in DESIGN.md: fits, dependency depth, segment frontier sizes, and
the solve's agreement with the serial raster-order evaluation of the same (centred) fits.

Every accepted fit t of every layer is x_t = c_t + sum_s beta_ts x_s (beta from the
weights and the integer offsets of the known window cells, value-independent; c_t the
solid sources).  Fits are ordered by (j + 5L, L, i) (a topological order); segments of K
consecutive fits each get their affine response to their frontier (earlier fits they read),
then one sequential pass over the segments applies the responses.

  python tools/pex_proto.py N [K] [steps_of_oracle_to_deform]
"""
import math
import sys
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fits_of(phi, dx, dy, layers):
    ny, nx = phi.shape
    known = phi < 0
    r2 = (4 * math.sqrt(dx * dx + dy * dy)) ** 2
    fits = []          # (L, j, i, [(jj, ii, beta)])
    acc_layer = -np.ones((ny, nx), dtype=np.int64)   # layer a cell was accepted in, -1 solid/none
    for L in range(layers):
        kst = known.copy()
        tgt = np.zeros_like(known)
        for dj in (-1, 0, 1):
            for di in (-1, 0, 1):
                tgt[1:-1, 1:-1] |= kst[1 + dj:ny - 1 + dj, 1 + di:nx - 1 + di]
        tgt &= ~kst
        tgt[0, :] = tgt[-1, :] = tgt[:, 0] = tgt[:, -1] = False
        js, is_ = np.nonzero(tgt)
        if len(js) == 0:
            break
        for j, i in zip(js, is_):
            x0, y0 = dx * i, dy * j
            src = []
            A = np.zeros(6)
            for jj in range(max(0, j - 4), min(ny, j + 5)):
                for ii in range(max(0, i - 4), min(nx, i + 5)):
                    if not known[jj, ii]:
                        continue
                    xi, yi = dx * ii, dy * jj
                    d2 = (xi - x0) ** 2 + (yi - y0) ** 2
                    if not d2 <= r2:
                        continue
                    w = math.exp(-d2 / r2)
                    a0, a1, a2 = w * 1.0, w * xi, w * yi
                    A += [a0 * 1.0, a0 * xi, a0 * yi, a1 * xi, a1 * yi, a2 * yi]
                    src.append((jj, ii, w))
            if len(src) < 3:
                continue
            a00, a01, a02, a11, a12, a22 = A
            det = (a00 * (a11 * a22 - a12 * a12) - a01 * (a01 * a22 - a12 * a02)
                   + a02 * (a01 * a12 - a11 * a02))
            if not abs(det) > 1e-10:
                continue
            S = np.zeros(6)
            for jj, ii, w in src:
                a, b = ii - i, jj - j
                S += [w, w * a, w * b, w * a * a, w * a * b, w * b * b]
            S0, Sx, Sy, Sxx, Sxy, Syy = S
            c00, c01, c02 = Sxx * Syy - Sxy * Sxy, Sx * Syy - Sxy * Sy, Sx * Sxy - Sxx * Sy
            dc = S0 * c00 - Sx * c01 + Sy * c02
            y0c, y1c, y2c = c00 / dc, -c01 / dc, c02 / dc
            fits.append((L, j, i, [(jj, ii, w * (y0c + y1c * (ii - i) + y2c * (jj - j)))
                                   for jj, ii, w in src]))
            known[j, i] = True
            acc_layer[j, i] = L
    return fits, acc_layer


def main():
    N = int(sys.argv[1])
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    from oracle import oracle as O
    O.set_all_cores(True); O.set_threads(len(os.sched_getaffinity(0)))
    sim = O.SoftDisc(N, "lid")
    for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 0):
        sim.step()
    phi0 = sim.phi_of(sim.X1, sim.X2)
    m = (phi0 <= 0).astype(float)
    X1 = sim.X1 * m
    dx = dy = sim.dx
    fits, accL = fits_of(phi0, dx, dy, sim.layers)
    # chain order (j + 5L, L, i) or, per layer (--layered), (L, j, i)
    layered = os.environ.get("PEX_LAYERED", "1") == "1"
    key = (lambda t: (fits[t][0], fits[t][1], fits[t][2])) if layered else \
          (lambda t: (fits[t][1] + 5 * fits[t][0], fits[t][0], fits[t][2]))
    order = sorted(range(len(fits)), key=key)
    ch = {(fits[t][1], fits[t][2]): c for c, t in enumerate(order)}
    F = [fits[t] for t in order]
    n = len(F)
    dyn = []          # per fit: [(chain index of source, beta)]
    cst = np.zeros(n)
    depth = np.zeros(n, dtype=np.int64)
    maxback = 0
    for c, (L, j, i, src) in enumerate(F):
        d = []
        for jj, ii, b in src:
            if (jj, ii) in ch:
                s = ch[(jj, ii)]
                assert s < c, "chain order is not topological"
                d.append((s, b)); maxback = max(maxback, c - s)
            else:
                cst[c] += b * X1[jj, ii]
        dyn.append(d)
        depth[c] = 1 + max((depth[s] for s, _ in d), default=0)
    # serial forward substitution (the oracle's raster order, centred fits)
    xs = np.zeros(n)
    for c in range(n):
        xs[c] = cst[c] + sum(b * xs[s] for s, b in dyn[c])
    # segment-affine solve
    nseg = (n + K - 1) // K
    fsz = []
    coef = []
    fronts = []
    layer_of = np.array([f[0] for f in F])
    # segments: K consecutive fits, not crossing a layer boundary (layered order)
    bounds = []
    c = 0
    while c < n:
        e = min(n, c + K)
        if layered:
            e = min(e, int(np.searchsorted(layer_of, layer_of[c], side="right")))
        bounds.append((c, e)); c = e
    nseg = len(bounds)
    for g, (lo, hi) in enumerate(bounds):
        # layered: earlier layers are final before this layer's pass (static sources)
        fr = sorted({s for c in range(lo, hi) for s, _ in dyn[c]
                     if s < lo and (not layered or layer_of[s] == layer_of[lo])})
        pos = {s: k for k, s in enumerate(fr)}
        fsz.append(len(fr))
        M = np.zeros((hi - lo, len(fr) + 1))
        for c in range(lo, hi):
            row = np.zeros(len(fr) + 1); row[-1] = cst[c]
            for s, b in dyn[c]:
                if s in pos:
                    row[pos[s]] += b
                elif s >= lo:
                    row += b * M[s - lo]
                else:
                    row[-1] += b * xs[s]     # an earlier layer's final value (static here)
            M[c - lo] = row
        coef.append(M); fronts.append(fr)
    xp = np.zeros(n)
    for g, (lo, hi) in enumerate(bounds):
        f = np.array([xp[s] for s in fronts[g]] + [1.0])
        xp[lo:lo + len(coef[g])] = coef[g] @ f
    # live sets R_g (fits before segment g read by segments >= g, same layer) and the rows of
    # the state transfer s_{g+1} = T_g s_g + e_g computed from segment g's outputs
    live, comp = [], []
    for g, (lo, hi) in enumerate(bounds):
        later = set()
        for h in range(g, len(bounds)):
            if layer_of[bounds[h][0]] != layer_of[lo]:
                break
            later |= set(fronts[h])
        live.append(len([s for s in later if s < lo]))
        comp.append(len([s for s in later if lo <= s < hi]))
    live, comp = np.array(live), np.array(comp)
    print(f"live state |R_g|: mean {live.mean():.1f} max {live.max()}; "
          f"state rows computed per segment: mean {comp.mean():.1f} max {comp.max()}")
    fsz = np.array(fsz)
    print(f"N={N} fits={n} layers={sim.layers} depth={depth.max()} max chain distance={maxback}")
    print(f"K={K}: segments={nseg} frontier mean={fsz.mean():.1f} p99={np.percentile(fsz, 99):.0f} "
          f"max={fsz.max()} (>62: {(fsz > 62).sum()})")
    print(f"segment-affine vs serial forward substitution: max |dx| = {np.abs(xp - xs).max():.3e}")
    dsrc = np.array([len(d) for d in dyn])
    print(f"dynamic sources per fit: mean {dsrc.mean():.1f} max {dsrc.max()}; "
          f"all sources: mean {np.mean([len(f[3]) for f in F]):.1f}")


if __name__ == "__main__":
    main()
