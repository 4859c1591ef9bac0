"""The fused step's asynchronous path (dt and max |u|^2 on the device, per-step diagnostics in
a device ring read back every 64 steps; sim.hip rmt_sim_step) against its synchronous path
(a finite t_end: dt read back and clipped on the host every step).  Same kernels, same
arithmetic: bit-identical fields and diagnostics."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_async_step_matches_sync_bitwise(gpu):
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    a, b = soft_disc_in_lid_driven(128), soft_disc_in_lid_driven(128)
    a.step(70)                 # async; 70 > 64 records: one ring flush inside the call
    b.step(70, t_end=1e30)     # finite t_end: the synchronous path
    a.step(5)                  # a second call starts from a fresh max |u|^2 reduction
    b.step(5, t_end=1e30)
    da, db = a.diagnostics(), b.diagnostics()
    assert len(da["t"]) == len(db["t"]) == 75
    for k in da:
        np.testing.assert_array_equal(da[k], db[k], err_msg=k)
    for f in ("u", "v", "p", "X1", "X2", "phi", "J"):
        np.testing.assert_array_equal(a.get(f), b.get(f), err_msg=f)


def test_async_step_reports_nonfinite_velocity(gpu):
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    s = soft_disc_in_lid_driven(64)
    s.step(3)
    u = s.get("u")
    u[10, 10] = np.nan
    s.set_field("u", u)
    with pytest.raises(FloatingPointError):
        s.step(4)
    assert len(s.diagnostics()["t"]) == 3    # the failing step is not recorded


def _carry_off(sim):
    from pyrmt_amd import _lib as L
    L.check(L.lib().rmt_sim_set_carry(sim.h, 0), "rmt_sim_set_carry")


def _same(a, b):
    da, db = a.diagnostics(), b.diagnostics()
    for k in da:
        np.testing.assert_array_equal(da[k], db[k], err_msg=k)
    for f in ("u", "v", "p", "X1", "X2", "phi", "J"):
        np.testing.assert_array_equal(a.get(f), b.get(f), err_msg=f)


def test_carry_across_calls_bitwise(gpu):
    """rmt_sim_set_carry (the Python Simulation's default): a call's first step starts from
    the geometry, known plane and max |u|^2 partials the previous call's last step left --
    four calls of 3 steps == the same four calls without the carry == one call of 12."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    a, b, c = (soft_disc_in_lid_driven(256) for _ in range(3))
    _carry_off(b)
    for s in (a, b):           # one sim after the other: they share the size's context, and
        for _ in range(4):     # another sim's step on it would end the carry (by design)
            s.step(3)
    c.step(12)
    _same(a, b)
    _same(a, c)


def test_carry_invalidated_by_writes_and_workspace_reuse(gpu):
    """A field written between calls (set_field: rmt_sim_invalidate) and another user of the
    context's workspace between calls (an extrapolation on the same-size context) both end
    the carry: results equal the no-carry run's."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    from pyrmt_amd import functions as F
    a, b = soft_disc_in_lid_driven(256), soft_disc_in_lid_driven(256)
    _carry_off(b)
    for s in (a, b):
        s.step(4)
        s.set_field("u", 0.5 * s.get("u"))
        s.step(4)
        X1, X2, phi = s.get("X1"), s.get("X2"), s.get("phi")
        F.extrapolate_reference_map(X1, X2, phi, 1.0 / 255, 1.0 / 255, 3)
        s.step(4)
    _same(a, b)


def test_carry_with_a_kept_view_written_later(gpu):
    """A field() view kept across step() calls and written through later, with no
    invalidate(): while such a view is alive every step() starts from the fields as they are
    (simulation.py), so the results equal the no-carry run's."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    a, b = soft_disc_in_lid_driven(256), soft_disc_in_lid_driven(256)
    _carry_off(b)
    for s in (a, b):
        u = s.field("u")          # kept
        s.step(3)
        s.step(2)
        u.mul_(0.5)               # written through the old view, no invalidate()
        s.step(3)
        del u
        s.step(2)
    _same(a, b)


def test_carry_with_a_derived_view_written_later(gpu):
    """A slice of a field() view outlives the view itself and is written through later: the
    slice keeps the storage (and so the carry check) alive, so the results equal the
    no-carry run's (only the undecorated view was tracked)."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    a, b = soft_disc_in_lid_driven(256), soft_disc_in_lid_driven(256)
    _carry_off(b)
    for s in (a, b):
        inner = s.field("u")[1:-1, 1:-1]   # the view itself is collected at once
        s.step(3)
        s.step(2)
        inner.mul_(0.5)                    # written through the slice, no invalidate()
        s.step(3)
        del inner
        s.step(2)
    _same(a, b)


@pytest.mark.parametrize("toggle", ["parallel", "mode"])
def test_carry_dropped_on_extrapolation_mode_change(gpu, toggle):
    """Switching the extrapolation's configuration between step() calls (the parallel mode,
    rmt_extrap_set_parallel; the path mode, rmt_extrap_set_mode) ends the carried geometry:
    the next step runs the new configuration from scratch, bit-identical to a run with the
    carry off (the carried geometry was the old mode's)."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    from pyrmt_amd import functions as F
    def on():
        if toggle == "parallel":
            F.extrapolation_parallel(True)
        else:
            F.extrapolation_mode(1)
    def off():
        if toggle == "parallel":
            F.extrapolation_parallel(False)
        else:
            F.extrapolation_mode(0)
    a, b = soft_disc_in_lid_driven(256), soft_disc_in_lid_driven(256)
    _carry_off(b)
    try:
        for s in (a, b):
            off()
            s.step(3)
            on()
            s.step(3)
            off()
            s.step(3)
    finally:
        off()
    _same(a, b)
