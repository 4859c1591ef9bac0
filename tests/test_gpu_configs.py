"""GPU parity at the BASELINE configs' own sizes (BASELINE.json `configs`).

The fused device step (rmt_sim_step / rmt_mac_sim_step through the C ABI) against the oracle
(oracle/, pinned bit-exact to the reference's fixtures) on the same inputs:
  config 4  soft_disc_in_lid_driven N=4096, 2 fused steps (the bench workload) vs the live
            oracle: X1, X2 after step 1 bit-exact, everything after step 2 at stated bars;
  config 2  soft_disc_in_lid_driven N=256, 1000 steps: centroid / J trajectory;
  config 3  disc_in_taylor_green N=1024 WENO5 + SSP-RK3, 20 steps: KE, SE, dissipation,
            its running integral and the total energy (disc_in_taylor_green.py:226-243);
  config 5  mac_multi_disc_lid N=8192 (3 discs, seed 3), 2 steps vs the oracle's fixture
            (tests/golden/gen_oracle_large.py: ~90 s per oracle step at this size).
Bars: bit-exact where the arithmetic has no transcendental function and no FFT on the path
to the compared value; otherwise the stated tolerance.  The only sources of difference are
the device `sin` of the smoothed Heaviside (ocml vs glibc, <= 1 ulp) and the DCT (the LDS
Stockham FFT vs pocketfft), both ~1e-16 relative per step.
The oracle runs in all-cores mode here (same results bit for bit, OpenMP on every per-cell
loop) so each test stays well inside the GPU box's per-test time limit.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fast_oracle(oracle):
    oracle.set_threads(min(16, os.cpu_count() or 1))
    oracle.set_all_cores(True)
    yield oracle
    oracle.set_all_cores(False)


def _maxdiff(a, b):
    return float(np.max(np.abs(np.asarray(a) - np.asarray(b))))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


def test_config4_fused_step_N4096_vs_oracle(gpu, fast_oracle):
    """The bench workload: 2 fused steps at N=4096 against the oracle's loop body."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    N = 4096
    ref = fast_oracle.SoftDisc(N, "lid")
    sim = soft_disc_in_lid_driven(N)
    # the initial narrow-band extrapolation (GPU chain vs the serial oracle sweep)
    assert _sha(sim.get("X1")) == _sha(ref.X1) and _sha(sim.get("X2")) == _sha(ref.X2)
    r1 = ref.step()
    sim.step(1)
    # step 1 starts from rest: advection and extrapolation are exact (no transcendental
    # function before the map update), so the advected + extrapolated map is bit-exact
    np.testing.assert_array_equal(sim.get("X1"), ref.X1)
    np.testing.assert_array_equal(sim.get("X2"), ref.X2)
    u1, v1, p1 = (sim.get(k) for k in ("u", "v", "p"))
    for got, want in ((u1, ref.a), (v1, ref.b), (p1, ref.p)):
        assert _maxdiff(got, want) <= 1e-12 * max(1.0, np.abs(want).max())
    r2 = ref.step()
    sim.step(1)
    d = sim.diagnostics()
    for k, r in enumerate((r1, r2)):
        np.testing.assert_allclose(d["dt"][k], r["dt"], rtol=1e-13)
        np.testing.assert_allclose([d["cx"][k], d["cy"][k]], [r["cx"], r["cy"]], rtol=1e-6)  # north star
        np.testing.assert_allclose([d["cx"][k], d["cy"][k]], [r["cx"], r["cy"]], rtol=1e-13)  # achieved
        np.testing.assert_allclose([d["minJ"][k], d["maxJ"][k]], [r["minJ"], r["maxJ"]], rtol=1e-11)
    ex1, ex2 = _maxdiff(sim.get("X1"), ref.X1), _maxdiff(sim.get("X2"), ref.X2)
    eu = _maxdiff(sim.get("u"), ref.a) / max(1.0, np.abs(ref.a).max())
    ev = _maxdiff(sim.get("v"), ref.b) / max(1.0, np.abs(ref.a).max())
    ep = _maxdiff(sim.get("p"), ref.p) / max(1.0, np.abs(ref.p).max())
    print(f"\n[config4 N=4096] step 2: |dX1| {ex1:.3g} |dX2| {ex2:.3g} |du| {eu:.3g} "
          f"|dv| {ev:.3g} |dp| {ep:.3g}")
    assert max(ex1, ex2) <= 1e-13          # measured 0 (bit-exact) on MI355X
    assert max(eu, ev) <= 1e-15 and ep <= 1e-12   # measured 9e-17, 6e-17, 1.9e-14


def test_config4_N4096_20_steps(gpu, fast_oracle):
    """The bench workload, 20 fused steps against the oracle: the per-step centroid at the
    north-star bar, minJ / maxJ within twice the reference's own noise floor at this size
    (1-ulp weight nudges of the oracle move them by up to 3.1e-4 / 6.1e-4 in 30 steps and the
    centroid by 4.8e-7: tools/noise_floor.py, profiles/r03/noise/lid_n4096.json)."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    N, S = 4096, 20
    ref = fast_oracle.SoftDisc(N, "lid")
    rec = [ref.step() for _ in range(S)]
    sim = soft_disc_in_lid_driven(N)
    sim.step(S)
    d = sim.diagnostics()
    keys = ("t", "cx", "cy", "minJ", "maxJ")
    want = np.array([[r[k] for k in keys] for r in rec])
    got = np.stack([d[k] for k in keys], axis=1)
    rel = np.abs(got - want) / np.abs(want)
    print(f"\n[config4 N=4096 x{S}] max rel: t {rel[:, 0].max():.3g} cx {rel[:, 1].max():.3g} "
          f"cy {rel[:, 2].max():.3g} minJ {rel[:, 3].max():.3g} maxJ {rel[:, 4].max():.3g}; "
          f"|dX1| {_maxdiff(sim.get('X1'), ref.X1):.3g} |du| {_maxdiff(sim.get('u'), ref.a):.3g}")
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-12)
    np.testing.assert_allclose(got[:, 1:3], want[:, 1:3], rtol=1e-6)     # north star
    np.testing.assert_allclose(got[:, 3], want[:, 3], rtol=7e-4)         # noise floor x 2
    np.testing.assert_allclose(got[:, 4], want[:, 4], rtol=1.3e-3)
    # achieved (MI355X): the map bit-exact after 20 steps, centroid 1.7e-15, J identical
    np.testing.assert_allclose(got[:, 1:3], want[:, 1:3], rtol=1e-12)
    np.testing.assert_allclose(got[:, 3:], want[:, 3:], rtol=1e-10)
    assert _maxdiff(sim.get("X1"), ref.X1) <= 1e-13 and _maxdiff(sim.get("X2"), ref.X2) <= 1e-13


def test_config2_N256_1000_steps(gpu, fast_oracle):
    """soft_disc_in_lid_driven N=256 (semi-Lagrangian): the per-step centroid / J trajectory
    (soft_disc_in_lid_driven.py:233) over 1000 steps."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    N, S = 256, 1000
    ref = fast_oracle.SoftDisc(N, "lid")
    rec = [ref.step() for _ in range(S)]
    sim = soft_disc_in_lid_driven(N)
    sim.step(S)
    d = sim.diagnostics()
    want = np.array([[r[k] for k in ("t", "cx", "cy", "minJ", "maxJ")] for r in rec])
    got = np.stack([d[k] for k in ("t", "cx", "cy", "minJ", "maxJ")], axis=1)
    rel = np.abs(got - want) / np.abs(want)
    print(f"\n[config2 N=256 x{S}] max rel: t {rel[:, 0].max():.3g} cx {rel[:, 1].max():.3g} "
          f"cy {rel[:, 2].max():.3g} minJ {rel[:, 3].max():.3g} maxJ {rel[:, 4].max():.3g}; "
          f"|dX1| {_maxdiff(sim.get('X1'), ref.X1):.3g} |du| {_maxdiff(sim.get('u'), ref.a):.3g}")
    np.testing.assert_allclose(got[:, 1:3], want[:, 1:3], rtol=1e-6)     # north star
    np.testing.assert_allclose(got[:, 0], want[:, 0], rtol=1e-12)
    np.testing.assert_allclose(got[:, 1:3], want[:, 1:3], rtol=1e-12)    # achieved
    # J min / max come from gradients of the band map, which amplifies the last-bit
    # differences of the smoothed Heaviside's sin; the reference's own noise floor for 1-ulp
    # perturbations is ~3e-9 after 388 steps at N=128
    np.testing.assert_allclose(got[:, 3:], want[:, 3:], rtol=1e-7)


def test_config3_N1024_weno5_energies(gpu, fast_oracle):
    """disc_in_taylor_green N=1024, WENO5 + SSP-RK3: per-step KE, SE, dissipation, its
    integral, total energy E (the drift check of disc_in_taylor_green.py:249-250), r_y, J."""
    from pyrmt_amd.simulation import disc_in_taylor_green
    N, S = 1024, 20
    ref = fast_oracle.SoftDisc(N, "tg", "weno5")
    rec = [ref.step(energies=True) for _ in range(S)]
    sim = disc_in_taylor_green(N, "weno5")
    sim.step(S)
    d = sim.diagnostics()
    keys = ("t", "ke", "se", "diss", "integ", "ry", "minJ")
    want = np.array([[r[k] for k in keys] + [r["E"]] for r in rec])
    got = np.stack([d[k] for k in keys] + [d["ke"] + d["se"] + d["integ"]], axis=1)
    rel = np.abs(got - want) / np.abs(want)
    print(f"\n[config3 N=1024 x{S}] max rel per column {dict(zip(keys + ('E',), rel.max(0)))}")
    drift = (got[-1, 7] - got[0, 7]) / got[0, 7]
    drift_ref = (want[-1, 7] - want[0, 7]) / want[0, 7]
    print(f"  energy drift over {S} steps: gpu {drift:.6e} oracle {drift_ref:.6e}")
    # north star: the energies (KE, dissipation and its integral, total E) within 1e-6
    col = {k: i for i, k in enumerate(keys + ("E",))}
    for k in ("ke", "diss", "integ", "E"):
        np.testing.assert_allclose(got[:, col[k]], want[:, col[k]], rtol=1e-6)
    # achieved (measured on MI355X: t, r_y exact; KE 1.1e-12; E 5.6e-9; dissipation 2.4e-8;
    # J 5e-8).  WENO5's smoothness weights and the band fits (Cramer on absolute coordinates,
    # 1-ulp noise -> 1e-9 at N=1024) amplify the last-bit differences of
    # the Heaviside's sin; SE = sum (mu/2)(I1 - 2) is ~1e-7 and crosses zero, so it is
    # compared in absolute terms against the energy scale (measured 1.4e-10).
    np.testing.assert_array_equal(got[:, col["t"]], want[:, col["t"]])
    np.testing.assert_allclose(got[:, col["ke"]], want[:, col["ke"]], rtol=1e-11)
    np.testing.assert_allclose(got[:, col["E"]], want[:, col["E"]], rtol=1e-7)
    np.testing.assert_allclose(got[:, col["diss"]], want[:, col["diss"]], rtol=1e-6)
    np.testing.assert_allclose(got[:, col["minJ"]], want[:, col["minJ"]], rtol=1e-6)
    assert np.abs(got[:, col["se"]] - want[:, col["se"]]).max() <= 1e-8 * np.abs(want[:, col["E"]]).max()
    assert abs(drift - drift_ref) <= 1e-8     # measured 1.4e-9 (drift itself -1.7e-4)


def test_config5_mac_N8192_vs_oracle_fixture(gpu):
    """mac_multi_disc_lid N=8192, 3 discs (seed 3): 2 steps against the oracle fixture."""
    from pyrmt_amd.mac import MacMultiDisc
    g = golden("mac8192_oracle")
    N, st = int(g["N"]), int(g["stride"])
    sim = MacMultiDisc(N, n_discs=3, seed=3)
    np.testing.assert_array_equal(np.array(sim.specs), g["specs"])
    assert sim.dt == float(g["dt"])
    worst = {}
    for s in (1, 2):
        sim.step(1)
        for k in range(3):
            jc, ic = g[f"rowcol_d{k}"]
            for name in ("X1", "X2", "phi"):
                f = sim.get(name, k)
                key = f"{name}_d{k}_s{s}"
                if s == 1:   # from rest: the maps are exact (no sin / DCT upstream)
                    assert _sha(f) == str(g[key + "_sha"]), key
                e = max(_maxdiff(f[jc], g[key + "_row"]), _maxdiff(f[:, ic], g[key + "_col"]),
                        _maxdiff(f[::st, ::st], g[key + "_sub"]))
                worst[key] = e
                assert e <= 1e-12, (key, e)
        for name in ("u", "v", "p"):
            want = g[f"{name}_s{s}"]
            got = sim.get(name)[::st, ::st]
            e = _maxdiff(got, want) / max(1.0, np.abs(want).max())
            worst[f"{name}_s{s}"] = e
            assert e <= 1e-10, (name, s, e)
    d = sim.diagnostics()
    gd = g["diag"]
    got = np.concatenate([np.stack([d["t"], d["dt"], d["minJ"], d["maxJ"]], 1), d["cx"], d["cy"]], 1)
    print(f"\n[config5 N=8192] worst field diffs {max(worst.values()):.3g}; diag max rel "
          f"{np.max(np.abs(got - gd) / np.abs(gd)):.3g}")
    np.testing.assert_allclose(got, gd, rtol=1e-6)      # north star
    np.testing.assert_allclose(got, gd, rtol=1e-12)     # achieved


def test_config5_schedule_switches_are_bit_identical(gpu):
    """N=8192, 3 discs: no first-layer fit is acceptable (det ~ 1e-14), so every extrapolation
    call is the identity.  The default reads k_ex_none's verdict back and launches nothing
    more (mac_noop_host); with it off every pass is launched and exits on the device flag.
    The advection samples the face planes (mac_face_sl) instead of centre planes a separate
    pass writes.  Defaults and both switches off must give the same bits over 3 steps."""
    import gc
    from pyrmt_amd.mac import MacMultiDisc
    out = []
    for opts in ({}, {"mac_noop_host": 0, "mac_face_sl": 0, "mac_m2_bound": 0}):
        sim = MacMultiDisc(8192, n_discs=3, seed=3, options=opts or None)
        sim.step(3)
        d = sim.diagnostics()
        out.append((d, {f"{n}{k}": _sha(sim.get(n, k)) for n in ("X1", "X2", "phi")
                        for k in range(3)} | {n: _sha(sim.get(n)) for n in ("u", "v", "p")}))
        del sim
        gc.collect()
    (d0, f0), (d1, f1) = out
    assert f0 == f1
    for k in d0:
        np.testing.assert_array_equal(d0[k], d1[k], err_msg=k)


def _diag100(sim):
    d = sim.diagnostics()
    return np.stack([d[k] for k in ("t", "dt", "cx", "cy", "minJ", "maxJ")], axis=1)


def test_config4_N4096_100_steps_vs_fixture(gpu):
    """The bench workload at the bench's length: 100 fused steps at N=4096 against the oracle's
    100-step fixture (tests/golden/gen_config4_100.py; soft_disc_in_lid_driven.py:206-235):
    the per-step t, dt, centroid and J range, and the final fields."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    g = golden("lid4096_100_oracle")
    N, S, st = int(g["N"]), int(g["steps"]), int(g["stride"])
    sim = soft_disc_in_lid_driven(N)
    sim.step(S)
    got, want = _diag100(sim), g["diag"]
    rel = np.abs(got - want) / np.abs(want)
    jc, ic = g["rowcol"]
    fd = {}
    for name in ("X1", "X2", "u", "v", "p", "phi"):
        f = sim.get(name)
        fd[name] = max(_maxdiff(f[::st, ::st], g[name + "_sub"]), _maxdiff(f[jc], g[name + "_row"]),
                       _maxdiff(f[:, ic], g[name + "_col"]))
        fd[name + "_sha"] = _sha(f) == str(g[name + "_sha"])
    print(f"\n[config4 N=4096 x{S}] max rel: t {rel[:, 0].max():.3g} dt {rel[:, 1].max():.3g} "
          f"cx {rel[:, 2].max():.3g} cy {rel[:, 3].max():.3g} minJ {rel[:, 4].max():.3g} "
          f"maxJ {rel[:, 5].max():.3g}; final fields {fd}")
    np.testing.assert_allclose(got[:, 2:4], want[:, 2:4], rtol=1e-6)     # north star
    np.testing.assert_allclose(got[:, 0:2], want[:, 0:2], rtol=1e-12)
    np.testing.assert_allclose(got[:, 4], want[:, 4], rtol=7e-4)         # noise floor x 2
    np.testing.assert_allclose(got[:, 5], want[:, 5], rtol=1.3e-3)
    # achieved (MI355X, round 4): t, dt and the J range equal, centroid
    # 1.7e-15, the map and phi equal on the sampled rows / columns / subgrid, u and v to
    # 2.2e-16, p to 1.1e-12 (the DCT's rounding against pocketfft's)
    np.testing.assert_allclose(got[:, 2:4], want[:, 2:4], rtol=1e-14)
    np.testing.assert_allclose(got[:, 4:6], want[:, 4:6], rtol=1e-14)
    assert max(fd["X1"], fd["X2"], fd["phi"]) <= 1e-14
    assert max(fd["u"], fd["v"]) <= 1e-14 and fd["p"] <= 1e-11


def test_config4_N4096_100_steps_parallel_mode(gpu):
    """The opt-in parallel extrapolation (extrap_par.hip: the reference's fits evaluated in
    centred coordinates) over the bench's 100 steps against the same oracle fixture.  It is
    not bit-exact.  Its bar is the reference's own noise floor over the same 100 steps at
    N=4096 (profiles/r05/noise/lid_n4096_100.json, tools/noise_floor.py): a 1-ulp nudge of
    the fit weights moves the reference's centroid by up to 5.78e-7 (cy, step 5), and the
    reference evaluated in centred coordinates on the CPU -- this mode's arithmetic -- lands
    1.147e-6 away, the same as this GPU mode.  Asserted: within twice the 1-ulp floor on
    every one of the 100 steps."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    g = golden("lid4096_100_oracle")
    N, S = int(g["N"]), int(g["steps"])
    gpu.extrapolation_parallel(True)
    try:
        sim = soft_disc_in_lid_driven(N)
        sim.step(S)
        got = _diag100(sim)
    finally:
        gpu.extrapolation_parallel(False)
    want = g["diag"]
    rel = np.abs(got - want) / np.abs(want)
    cen = rel[:, 2:4].max(axis=1)
    past = np.nonzero(cen > 1e-6)[0]
    first = int(past[0]) + 1 if len(past) else None
    print(f"\n[config4 N=4096 x{S}, parallel extrapolation] worst centroid rel {cen.max():.3g} "
          f"(step {int(cen.argmax()) + 1}); first step past 1e-6: {first}; t {rel[:, 0].max():.3g} "
          f"minJ {rel[:, 4].max():.3g} maxJ {rel[:, 5].max():.3g}")
    floor = 5.781624386615219e-07   # lid_n4096_100.json: nudge_1ulp, max of cx / cy max_rel
    # (2 x floor = 1.156e-6 was chosen with this mode's 1.147e-6 already measured: it pins the
    # measured state, it does not qualify the mode -- north_star's bar is 1e-6, which the mode
    # holds for the first 20 steps only, asserted separately)
    assert np.all(cen <= 2 * floor), (cen.max(), int(cen.argmax()) + 1)
    assert np.all(cen[:20] <= 1e-6), (cen[:20].max(), int(cen[:20].argmax()) + 1)
    # the J range against the reference's 1-ulp floor over the same 100 steps (nudge_1ulp:
    # minJ 3.146e-4, maxJ 6.092e-4 max_rel): minJ stays within twice it (6.08e-4 measured, the
    # CPU centred evaluation), maxJ does not -- 3.52e-3, 5.8 x the floor:
    # asserted at the measured level so that a regression shows, and recorded as a gap
    jfloor_min, jfloor_max = 3.1461450124562043e-04, 6.091788058037263e-04
    assert rel[:, 4].max() <= 2 * jfloor_min, rel[:, 4].max()
    assert rel[:, 5].max() <= 6 * jfloor_max, rel[:, 5].max()
