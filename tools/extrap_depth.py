"""Dependency depth of the exact extrapolation chain (functions.py:48-163) for a test case:
the longest path, in fits, when each fit costs one unit, a row's targets run in order on one
wave, row (L, j) waits for rows j-4..j+4 of layer L-1 and for rows j-1..j-4 of layer L to pass
column i+4 (k_ex_sweep's rule), and tickets go to NW waves in order of j + 5L.
    python tools/extrap_depth.py disc4096 8 1   # case, waves, per-row overhead (fits)"""
import sys, heapq, numpy as np
sys.path.insert(0,'/root/repo/tests'); sys.path.insert(0,'/root/repo')
from test_gpu_parity import _extrap_case
from scipy.ndimage import binary_dilation
name=sys.argv[1]; NW=int(sys.argv[2]); crow=float(sys.argv[3])
X1,X2,phi,dx,dy,ML=_extrap_case(name)
ny,nx=phi.shape
known=phi<0
interior=np.zeros_like(known); interior[1:-1,1:-1]=True
layers=[]
for L in range(ML):
    tgt=(~known)&binary_dilation(known,structure=np.ones((3,3),bool))&interior
    layers.append(tgt); known=known|tgt
rows={}
for L in range(ML):
    for j in range(ny):
        c=np.nonzero(layers[L][j])[0]
        if len(c): rows[(L,j)]=c
jl=min(j for _,j in rows); jh=max(j for _,j in rows)
# tickets
tickets=[]
for k in range(jl, jh+5*(ML-1)+1):
    for L in range(ML):
        j=k-5*L
        if jl<=j<=jh: tickets.append((L,j))
fin={}  # (L,j) -> list of finish times per target
done_row={}
# discrete simulation: waves process tickets in order; a ticket's targets need deps
# compute greedily in ticket order with wave availability
import collections
wave_free=[0.0]*NW
heapq.heapify(wave_free)
def row_done(L,j):
    if (L,j) not in rows: return 0.0
    return done_row[(L,j)]
for (L,j) in tickets:
    t0=heapq.heappop(wave_free)   # wave takes next ticket when free
    if (L,j) not in rows:
        heapq.heappush(wave_free,t0); done_row[(L,j)]=t0; continue
    t=t0+crow
    if L>0:
        for r in range(-4,5):
            if (L-1,j+r) in rows: t=max(t,done_row[(L-1,j+r)])
    cols=rows[(L,j)]; f=np.zeros(len(cols))
    for k,i in enumerate(cols):
        for r in range(1,5):
            if (L,j-r) in rows:
                c2=rows[(L,j-r)]; m=c2<=i+4
                if m.any(): t=max(t,fin[(L,j-r)][m].max())
        t=t+1; f[k]=t
    fin[(L,j)]=f; done_row[(L,j)]=t
    heapq.heappush(wave_free,t)
print(name,"waves",NW,"rowcost",crow,"makespan",max(done_row.values()))
