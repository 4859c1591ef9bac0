"""Latency model of the exact extrapolation chain (functions.py:48-163) on the bench state.

For every fit of the N=4096 soft-disc band (3 layers): its included window cells in window
order, which of them are values an earlier fit produces (dynamic) and the fit that produces
each.  A fit's critical path after its last-arriving source is: hand-off of that value + the
ordered fold of every term after its window position + the 3x3 solve.  This script computes
the makespan (infinite waves) under a cycle model, to size the chain kernel's design choices:
    python tools/chain_model.py [N] [c_add] [c_solve] [c_handoff] [c_same_wave]
"""
import sys

import numpy as np
from scipy.ndimage import binary_dilation

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
C_ADD, C_SOLVE, C_H, C_SAME = (float(a) for a in (sys.argv[2:6] + ["8", "100", "250", "20"][len(sys.argv[2:6]):]))

x = np.linspace(0.0, 1.0, N)
dx = x[1] - x[0]
X, Y = np.meshgrid(x, x)
phi = np.sqrt((X - 0.6) ** 2 + (Y - 0.5) ** 2) - 0.2
known0 = phi < 0
r = 4 * np.sqrt(dx * dx + dx * dx)
r2 = r * r
ML = 3
interior = np.zeros_like(known0)
interior[1:-1, 1:-1] = True

# window offsets included by the radius test (same float ops as the reference, at a
# representative cell; the included set is translation-invariant up to rounding)
offs = []
for dj in range(-4, 5):
    for di in range(-4, 5):
        i0, j0 = N // 2, N // 2
        ddx = dx * (i0 + di) - dx * i0
        ddy = dx * (j0 + dj) - dx * j0
        if ddx * ddx + ddy * ddy <= r2:
            offs.append((dj, di))

known = known0.copy()
fid = -np.ones((N, N), dtype=np.int64)       # fit id producing a cell (dynamic source)
fits = []                                     # (L, j, i)
for L in range(ML):
    tgt = (~known) & binary_dilation(known, structure=np.ones((3, 3), bool)) & interior
    js, is_ = np.nonzero(tgt)
    order = np.lexsort((is_, js))
    for k in order:
        j, i = int(js[k]), int(is_[k])
        fid[j, i] = len(fits)
        fits.append((L, j, i))
    known = known | tgt
nf = len(fits)
print(f"N={N}: {nf} fits, {len(offs)} window cells in radius")

# per fit: ordered list of (is_dynamic, source id) over included cells from the first dynamic
fin = np.zeros(nf)
tail_after_last_src = []
nd_hist = []
for t, (L, j, i) in enumerate(fits):
    terms = []
    for dj, di in offs:
        jj, ii = j + dj, i + di
        if not (0 <= jj < N and 0 <= ii < N):
            continue
        if known0[jj, ii]:
            terms.append(-1)
            continue
        s = fid[jj, ii]
        if s < 0:
            continue
        Ls = fits[s][0]
        # known at t's time: fitted in an earlier layer, or same layer and raster-earlier
        if Ls < L or (Ls == L and (jj < j or (jj == j and ii < i))):
            terms.append(s)
    dyn = [k for k, s in enumerate(terms) if s >= 0]
    nd_hist.append(len(dyn))
    if not dyn:
        fin[t] = C_SOLVE
        continue
    tm = 0.0
    for k in range(dyn[0], len(terms)):
        s = terms[k]
        if s >= 0:
            same = s == t - 1 and fits[s][0] == L and fits[s][1] == j
            tm = max(tm, fin[s] + (C_SAME if same else C_H))
        tm += C_ADD
    fin[t] = tm + C_SOLVE
    tail_after_last_src.append(len(terms) - 1 - max(dyn, key=lambda k: fin[terms[k]]))
mk = fin.max()
print(f"dynamic sources per fit: mean {np.mean(nd_hist):.1f} max {max(nd_hist)}; "
      f"fold terms after the latest source: mean {np.mean(tail_after_last_src):.1f}")
print(f"model c_add={C_ADD} c_solve={C_SOLVE} c_handoff={C_H} c_same={C_SAME}: makespan "
      f"{mk:.0f} cycles = {mk / 2.4e3:.3f} ms at 2.4 GHz")


# ---- finite wave pool: a wave takes the next fit in chain order when free and is busy
# until the fit is done (its pre-arrival work, the wait, the post-arrival fold + solve, the
# store); chain order = (j + 5L, L, i) as k_ex_order
def pool(W, c_pre, c_post_fixed, c_add, c_h, c_store):
    import heapq
    order = sorted(range(nf), key=lambda t: (fits[t][1] + 5 * fits[t][0], fits[t][0], fits[t][2]))
    free = [0.0] * W
    heapq.heapify(free)
    done = np.zeros(nf)
    for t in order:
        w0 = heapq.heappop(free)
        tm = w0 + c_pre
        for (k, s, after) in deps[t]:
            tm = max(tm, done[s] + c_h + after * c_add)
        done[t] = tm + c_post_fixed
        heapq.heappush(free, done[t] + c_store)
    return done.max()


# per fit: (position, source, number of terms after it) for its dynamic sources
deps = []
for t, (L, j, i) in enumerate(fits):
    terms = []
    for dj, di in offs:
        jj, ii = j + dj, i + di
        if not (0 <= jj < N and 0 <= ii < N):
            continue
        if known0[jj, ii]:
            terms.append(-1)
            continue
        s = fid[jj, ii]
        if s < 0:
            continue
        Ls = fits[s][0]
        if Ls < L or (Ls == L and (jj < j or (jj == j and ii < i))):
            terms.append(s)
    deps.append([(k, s, len(terms) - 1 - k) for k, s in enumerate(terms) if s >= 0])
for W, pre, post, add, h, st in ((24, 2800, 500, 20, 400, 500), (24, 1500, 150, 8, 150, 200),
                                 (24, 800, 120, 8, 120, 100), (48, 800, 120, 8, 120, 100),
                                 (12, 800, 120, 8, 120, 100)):
    mk = pool(W, pre, post, add, h, st)
    print(f"pool W={W} pre={pre} post={post} add={add} handoff={h} store={st}: "
          f"{mk / 2.4e6:.3f} ms")
