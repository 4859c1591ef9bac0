"""The rerun-after-overflow scenario of tests/test_distributed.py
(test_slab_rerun_after_late_dropped_geometry) with the dropped geometry NOT waited for
(test_nowait_drop=1, the behaviour before the wait in rmt_slab_drop_geometry): does a late
geometry landing inside the rerun's extrapolation break the run?  Prints one line per variant:
ok / mismatch / the error raised.  Diagnostic, run once.

    python tools/slab_drop_hazard.py [delay_units]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyrmt_amd import distributed as D  # noqa: E402
from pyrmt_amd.simulation import soft_disc_in_lid_driven  # noqa: E402

N, K = 256, 10
delay = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
ref = soft_disc_in_lid_driven(N)
ref.step(K)
want = {f: ref.get(f) for f in ("u", "v", "p", "X1", "X2")}
for opts in ({"test_delay_geo": delay, "test_nowait_drop": 1},
             {"test_delay_geo": delay}):
    try:
        sim = D.soft_disc_in_lid_driven(N, D.LocalComm(2), options=opts)
        sim.sync_every = 4
        sim.step(2)
        sim._rim_cap = 1
        sim.step(K - 2)
        bad = [f for f in want if not np.array_equal(sim.gather(f), want[f])]
        res = "ok" if not bad else "mismatch in " + ",".join(bad)
        res += f" (reruns {getattr(sim, 'reruns', 0)})"
    except Exception as e:  # noqa: BLE001 -- the outcome is what this probe reports
        res = f"{type(e).__name__}: {e}"
    print(opts, "->", res, flush=True)
