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
