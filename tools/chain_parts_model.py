"""Wave-pool model of the exact extrapolation chain (functions.py:95-161) under different
assignments of fits to chain workgroups ("parts"), to size the part split before building it.

Fits of the N=4096 soft-disc band (the bench geometry, 3 layers) in chain order (j + 5L, L, i).
A part is one workgroup of W waves taking its fits round robin in chain order; a fit occupies
its wave from its start (the wave's previous fit published + c_store) through c_pre of
pre-arrival work, the wait for its sources and the post-arrival work: for a source s at window
position k, the fit cannot publish before done[s] + hand-off + (terms after k) * c_add +
c_post.  The hand-off is c_local inside a part (LDS ring) and c_far across parts (8-byte
agent-scope granules through L2 / the fabric).

    python tools/chain_parts_model.py [N]
"""
import heapq
import sys

import numpy as np
from scipy.ndimage import binary_dilation

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ML = 3
x = np.linspace(0.0, 1.0, N)
dx = x[1] - x[0]
X, Y = np.meshgrid(x, x)
known0 = (np.sqrt((X - 0.6) ** 2 + (Y - 0.5) ** 2) - 0.2) < 0
r2 = (4 * np.sqrt(dx * dx + dx * dx)) ** 2
interior = np.zeros_like(known0)
interior[1:-1, 1:-1] = True
offs = []
for dj in range(-4, 5):
    for di in range(-4, 5):
        ddx = dx * (N // 2 + di) - dx * (N // 2)
        ddy = dx * (N // 2 + dj) - dx * (N // 2)
        if ddx * ddx + ddy * ddy <= r2:
            offs.append((dj, di))

known = known0.copy()
fid = -np.ones((N, N), dtype=np.int64)
fits = []
for L in range(ML):
    tgt = (~known) & binary_dilation(known, structure=np.ones((3, 3), bool)) & interior
    js, is_ = np.nonzero(tgt)
    for k in np.lexsort((is_, js)):
        j, i = int(js[k]), int(is_[k])
        fid[j, i] = len(fits)
        fits.append((L, j, i))
    known = known | tgt
nf = len(fits)
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
    deps.append([(s, len(terms) - 1 - k) for k, s in enumerate(terms) if s >= 0])
order = sorted(range(nf), key=lambda t: (fits[t][1] + 5 * fits[t][0], fits[t][0], fits[t][2]))
cols = np.array([f[2] for f in fits])
cmin, span = cols.min(), cols.max() - cols.min() + 1
print(f"N={N}: {nf} fits")


def run(part_of, W, c_pre=2000, c_post=550, c_add=20, c_local=370, c_far=2400, c_store=300):
    P = max(part_of) + 1
    free = [[0.0] * W for _ in range(P)]
    done = np.zeros(nf)
    far = 0
    for t in order:
        p = part_of[t]
        w0 = heapq.heappop(free[p])
        tm = w0 + c_pre
        for s, after in deps[t]:
            h = c_local if part_of[s] == p else c_far
            far += part_of[s] != p
            tm = max(tm, done[s] + h + after * c_add)
        done[t] = tm + c_post
        heapq.heappush(free[p], done[t] + c_store)
    return done.max() / 2.4e6, far


side = [int((f[2] - cmin) * 2 // span) for f in fits]
col2 = side
layer = [f[0] for f in fits]
side_layer = [s * ML + L for s, L in zip(side, layer)]
side_l01 = [s * 2 + min(L, 1) for s, L in zip(side, layer)]
for name, po in (("2 column parts", col2), ("side x layer (6)", side_layer),
                 ("side x {0},{1,2} (4)", side_l01)):
    for W in (8, 12, 16):
        ms, far = run(po, W)
        print(f"{name:22s} W={W:2d}: {ms:.3f} ms  (cross-part source reads {far})")
# link-latency sensitivity of the 6-part split
for c_add, c_post, c_local in ((20, 550, 370), (12, 400, 300), (8, 300, 250)):
    ms, _ = run(side_layer, 12, c_add=c_add, c_post=c_post, c_local=c_local)
    print(f"side x layer W=12 c_add={c_add} c_post={c_post} c_local={c_local}: {ms:.3f} ms")
# the tail fold taken off the link (residue-class folds before the arrival): a constant
# c_post instead of after * c_add
for c_post, c_local in ((650, 370), (500, 300), (400, 250)):
    for name, po in (("2 column parts", col2), ("side x layer (6)", side_layer)):
        ms, _ = run(po, 16, c_add=0, c_post=c_post, c_local=c_local)
        print(f"{name:22s} W=16 no tail fold, c_post={c_post} c_local={c_local}: {ms:.3f} ms")
