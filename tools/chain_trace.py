"""Critical-path analysis of a k_ex_chain trace (RMT_EX_PROFILE=1 RMT_EX_TRACE=path): per fit
{start, ready (all sources in), published, critical source slot, wave, cell} in
s_memrealtime ticks (10 ns).  Walks back from the last publish: a fit that waited for a source
continues at that source ("source" step), one whose sources were in before it started
continues at its wave's previous fit ("wave" step).
    python tools/chain_trace.py trace.bin [nx] [parts]"""
import sys
import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.int64).reshape(-1, 6)
nx = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
NP = int(sys.argv[3]) if len(sys.argv) > 3 else 2
n = len(t)
st, rd, pb, crit, wave, cell = (t[:, k].copy() for k in range(6))
ok = st > 0
t0 = st[ok].min()
col = cell % nx
cmin, span = col[ok].min(), col[ok].max() - col[ok].min() + 1
if (wave >> 8).max() > 0:   # round 5: wave | part << 8 (parts: column range x layer group)
    part = wave >> 8
    wave = wave & 255
else:
    part = np.minimum(NP - 1, np.maximum(0, (col - cmin) * NP // span))
print(f"{n} fits ({ok.sum()} traced); span {(pb.max() - t0) / 100:.1f} us; parts {np.bincount(part)}")
det = np.where((crit >= 0) & ok, rd - pb[np.maximum(crit, 0)], -1)
post = (pb - rd)
pre = (rd - st)
print(f"ready -> published: median {np.median(post[ok]) * 10:.0f} ns, mean {post[ok].mean() * 10:.0f} ns, "
      f"p90 {np.percentile(post[ok], 90) * 10:.0f} ns")
w = det >= 0
print(f"source published -> noticed (fits that waited): median {np.median(det[w]) * 10:.0f} ns, "
      f"mean {det[w].mean() * 10:.0f} ns  ({w.sum()} fits waited)")
# previous fit of the same (part, wave) by start time
prev = -np.ones(n, dtype=np.int64)
last = {}
for k in np.argsort(st):
    if not ok[k]:
        continue
    key = (int(part[k]), int(wave[k]))
    prev[k] = last.get(key, -1)
    last[key] = k
f = int(np.argmax(pb))
nsrc = nwave = 0
tsrc = twave = 0.0
seen = set()
postc, detc, gapw = [], [], []
while f >= 0 and f not in seen:
    seen.add(f)
    c = int(crit[f])
    if c >= 0 and rd[f] > st[f] and pb[c] >= st[f]:
        nsrc += 1; tsrc += pb[f] - pb[c]
        postc.append(post[f]); detc.append(rd[f] - pb[c])
        f = c
    else:
        p = int(prev[f])
        nwave += 1; twave += pb[f] - (pb[p] if p >= 0 else t0)
        gapw.append(st[f] - (pb[p] if p >= 0 else t0))
        f = p
print(f"critical path: {nsrc} source steps ({tsrc / 100:.0f} us, {tsrc * 10 / max(nsrc, 1):.0f} ns each: "
      f"detect {np.mean(detc) * 10:.0f} + post {np.mean(postc) * 10:.0f}), "
      f"{nwave} wave steps ({twave / 100:.0f} us, {twave * 10 / max(nwave, 1):.0f} ns each, "
      f"{np.mean(gapw) * 10 if gapw else 0:.0f} ns of it before the start)")

# geometry of the critical-path source steps: (row, column) offset of the critical source
f = int(np.argmax(pb))
seen = set()
offs = {}
while f >= 0 and f not in seen:
    seen.add(f)
    c = int(crit[f])
    if c >= 0 and rd[f] > st[f] and pb[c] >= st[f]:
        dj = int(cell[f] // nx - cell[c] // nx); di = int(cell[f] % nx - cell[c] % nx)
        offs[(dj, di)] = offs.get((dj, di), 0) + 1
        f = c
    else:
        f = int(prev[f])
tot = sum(offs.values())
print("critical source offsets (dj, di): " + ", ".join(
    f"{k}: {v * 100 / tot:.0f}%" for k, v in sorted(offs.items(), key=lambda kv: -kv[1])[:10]))
