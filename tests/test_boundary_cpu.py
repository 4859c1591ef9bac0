"""CPU-side checks of the drop-in boundary: librmt.so loads without a GPU and exports
every entry point include/rmt.h declares; the Python shim binds each of them; host
logic (BC / shape descriptors) matches the reference drivers' callables."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "rmt.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(rmt_\w+)\(", src, re.M)))


def test_header_symbols_exported():
    from pyrmt_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build librmt.so first (__graft_entry__.build())"
    h = ctypes.CDLL(_lib.LIB_PATH)
    names = _declared()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(h, n)]
    assert not missing, missing
    unbound = [n for n in names if n not in _lib.SIGNATURES]
    assert not unbound, unbound


def test_library_loads_and_reports_version():
    import pyrmt_amd
    lib = pyrmt_amd.library()
    assert lib.rmt_version() == 1
    assert lib.rmt_last_error() is not None


def _no_slip_lid_bc(u, v, lid_speed=1.0):
    u = u.copy(); v = v.copy()
    u[:, 0] = 0.0; v[:, 0] = 0.0; u[:, -1] = 0.0; v[:, -1] = 0.0
    u[0, :] = 0.0; v[0, :] = 0.0; u[-1, :] = lid_speed; v[-1, :] = 0.0
    u[0, 0] = u[0, -1] = u[-1, 0] = u[-1, -1] = 0.0
    v[0, 0] = v[0, -1] = v[-1, 0] = v[-1, -1] = 0.0
    return u, v


def _free_slip_box_bc(u, v):
    u = u.copy(); v = v.copy()
    u[:, 0] = 0.0; u[:, -1] = 0.0
    v[:, 0] = v[:, 1]; v[:, -1] = v[:, -2]
    v[0, :] = 0.0; v[-1, :] = 0.0
    u[0, :] = u[1, :]; u[-1, :] = u[-2, :]
    return u, v


def test_bc_descriptors_match_reference_callables(oracle):
    from pyrmt_amd.bc import NoSlipLid, FreeSlipBox, resolve_bc
    rng = np.random.default_rng(0)
    u, v = rng.standard_normal((2, 11, 13))
    for desc, ref, kind in ((NoSlipLid(2.5), lambda a, b: _no_slip_lid_bc(a, b, 2.5), 1),
                            (FreeSlipBox(), _free_slip_box_bc, 2)):
        du, dv = desc(u, v)
        ru, rv = ref(u, v)
        np.testing.assert_array_equal(du, ru); np.testing.assert_array_equal(dv, rv)
        assert resolve_bc(ref)[0] == kind
        ou, ov = oracle.apply_bc(kind, desc.lid, u, v)        # the oracle's C BC too
        np.testing.assert_array_equal(ou, ru); np.testing.assert_array_equal(ov, rv)
    with pytest.raises(NotImplementedError):
        resolve_bc(lambda a, b: (a * 2, b))


def test_disc_shape_probe():
    from pyrmt_amd.bc import resolve_shape, Disc
    for x0, y0, R in ((0.6, 0.5, 0.2), (0.5, 0.5, 0.2), (0.37, 0.61, 0.113)):
        d = resolve_shape(lambda X, Y: np.sqrt((X - x0) ** 2 + (Y - y0) ** 2) - R)
        assert (d.x0, d.y0, d.R) == (x0, y0, R)
    assert isinstance(resolve_shape(Disc(0.1, 0.2, 0.3)), Disc)
    with pytest.raises(NotImplementedError):
        resolve_shape(lambda X, Y: X + Y)
