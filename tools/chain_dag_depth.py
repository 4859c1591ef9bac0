"""Dependency depth of the exact extrapolation chain (functions.py:95-161: raster order within
a layer, each accepted fit known at once) on the bench state's band (the N=4096 soft disc,
3 layers; tools/chain_parts_model.py builds the fits and their window sources): the longest
chain of fits each reading the previous one's value.  The chain kernel cannot finish in fewer
hand-offs than this; bench.py reports the chain's time per link on it.

    python tools/chain_dag_depth.py [N] [OUT.json]
"""
import json
import os
import sys

import numpy as np

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
out = sys.argv[2] if len(sys.argv) > 2 else None
here = os.path.dirname(os.path.abspath(__file__))
src = open(os.path.join(here, "chain_parts_model.py")).read()
src = src[:src.index("side = [")]          # the fits, their sources and the chain order only
sys.argv = [sys.argv[0], str(N)]
exec(src)
hop = np.zeros(nf, dtype=np.int64)
for t in order:
    hop[t] = max((hop[s] + 1 for s, _ in deps[t]), default=0)
per_layer = {}
for L in range(ML):
    idx = [t for t in range(nf) if fits[t][0] == L]
    per_layer[str(L)] = {"fits": len(idx), "depth": int(hop[idx].max())}
res = {"N": N, "layers": ML, "fits": nf, "depth": int(hop.max()), "per_layer": per_layer,
       "state": "the driver's initial disc (0.6, 0.5, 0.2); tools/chain_parts_model.py"}
print(json.dumps(res))
if out:
    json.dump(res, open(out, "w"), indent=1)
