"""k_ex_chain time (HIP events around the chain launch) on the bench-size disc, per
RMT_CH_VARIANT value given on the command line (each in a fresh process).
    python tools/chain_time.py [variant ...]"""
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 1 and sys.argv[1] == "--one":
    sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
    import numpy as np
    import pyrmt_amd as P
    from pyrmt_amd import _lib as L, functions as F
    from test_gpu_parity import _extrap_case
    X1, X2, phi, dx, dy, layers = _extrap_case("disc4096")
    ref = P.extrapolate_reference_map(X1, X2, phi, dx, dy, layers)
    c = F.ctx_for(*phi.shape)
    L.check(L.lib().rmt_ctx_set_profiling(c.h, 1))
    ms = []
    for _ in range(5):
        g = P.extrapolate_reference_map(X1, X2, phi, dx, dy, layers)
        m2 = (ctypes.c_double * 2)()
        L.check(L.lib().rmt_ctx_kernel_ms(c.h, m2))
        ms.append(m2[1])
    ok = np.array_equal(g[0], ref[0]) and np.array_equal(g[1], ref[1])
    print(f"variant {os.environ.get('RMT_CH_VARIANT', '0')}: chain {min(ms):.3f} ms "
          f"(median {sorted(ms)[2]:.3f}) path {P.extrapolation_last_path(*phi.shape)} same={ok}")
    sys.exit(0)
for v in sys.argv[1:] or ["0"]:
    env = dict(os.environ, RMT_CH_VARIANT=v)
    subprocess.run([sys.executable, os.path.abspath(__file__), "--one"], env=env, check=True,
                   timeout=300)
