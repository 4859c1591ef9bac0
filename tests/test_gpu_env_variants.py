"""The fused step's schedule and kernel switches (rmt_ctx_set_option: per-context
implementation switches, include/rmt.h) against the default: every one reorders or overlaps
the same kernels, or computes the same arithmetic another way, so fields and diagnostics must
be bit-identical.  N=256 so that the split projection (LDS DCT plan:
255 = 3 5 17) and with it the early transpose are on.  Each variant runs in this process on
a context of its own (Simulation(options=...)); one child process checks that the
environment variables still set a new context's defaults.

  sim_hiprio=0          the step on the caller's stream instead of the highest-priority one
  early_transpose=0     the column pass's transpose entirely after the chain
  early_geometry=0      the next step's extrapolation geometry on the main stream
  side_tail=0           p -= mean(p) and the diagnostics right after the projection
  no_overlap=1          no second stream at all
  sim_sync=1            dt read back on the host every step
  chain_cols=1 / 4      the chain's column ranges (x layer groups: more cross-part hand-offs)
  chain_layer_groups=1  all layers of a column range in one workgroup (round 4's parts)
  fused_fluid=0         the momentum's pure-fluid flags from their own pass over phi
  ex mode 2             the extrapolation's forced fallback sweep, which the fused step runs
                        on its second stream beside the chain (functions.extrapolation_mode)
  fused_fixprep=0       the fix-up's phi and momentum prep in two kernels (the sweep in order)
  ext_events=0          the cross-stream events recorded after their kernels instead of
                        completing with them (hipExtLaunchKernel)
  merged_join=0         the second stream joined twice (after its momentum, before the
                        projection) instead of once after its row passes
  test_delay_side=300   the second stream sleeps ~1 ms as its work beside the chain starts
  test_delay_main=300   the critical stream sleeps ~1 ms right after the chain (both: every
                        cross-stream read is ordered by an event, whatever the timing)
  fix_all=1             the fix-up re-runs phi, the prep and the four stages on EVERY tile
                        (interior, edge and domain-boundary tiles through the list kernels;
                        the default's fix-up list holds interior tiles only for this disc) --
                        the regression test for the round-3 divergent list-kernel variant
                        
  transpose2=0          the 8-byte transposes
  edge_stream=0         a full stage's edge tiles after its interior launch on the same stream
                        instead of beside it on a stream of their own
  sl_phi=0              phi, the known-plane words and the fluid flags from k_phi_rebuild_fluid
                        after the side stream's SL pass instead of from that pass itself
  skip_marked_rows=0    the speculative row DCT also transforms the rows the fix-up transforms
                        again afterwards
  tail_stream=0         the pressure update (p + (pc - m), p -= mean p) on the second stream
                        ahead of its SL pass instead of beside it on the edge-tile stream
  diag_first=1          the step's diagnostics ahead of the next step's geometry instead of
                        behind it
  sl_zero_flags=0       the second stream's SL pass loads and stores every tile instead of
                        skipping the tiles its zero-tile flags prove +0.0

Every variant above runs the diagnostics through k_diag_seg (its segment skip adds nothing to
any lane's sums, so the skip pattern does not change the bits).  diag_seg=0 (k_diag_p1's
strided visit order: the same terms summed in another order) is compared separately:
fields and J extrema exact, the centroid to rounding.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("u", "v", "p", "X1", "X2", "phi", "J")


def _run(options=None, ex_mode=None):
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    from pyrmt_amd.functions import extrapolation_mode
    if ex_mode is not None:
        extrapolation_mode(ex_mode)
    try:
        s = soft_disc_in_lid_driven(256, options=options)
        s.step(12)
        out = {f: s.get(f) for f in FIELDS}
        out.update({"d_" + k: np.asarray(v) for k, v in s.diagnostics().items()})
    finally:
        if ex_mode is not None:
            extrapolation_mode(0)
    return out


@pytest.fixture(scope="module")
def default_run(gpu):
    return _run()


def _same(got, ref):
    assert sorted(got) == sorted(ref)
    for k in ref:
        np.testing.assert_array_equal(got[k], ref[k], err_msg=k)


@pytest.mark.parametrize("opts", [
    {"sim_hiprio": 0}, {"early_transpose": 0}, {"early_geometry": 0},
    {"side_tail": 0}, {"no_overlap": 1}, {"sim_sync": 1},
    {"chain_cols": 1}, {"chain_cols": 4}, {"chain_layer_groups": 1},
    {"chain_cols": 1, "chain_layer_groups": 1}, {"fused_fluid": 0},
    {"fused_fixprep": 0}, {"ext_events": 0}, {"transpose2": 0},
    {"merged_join": 0}, {"test_delay_side": 300}, {"test_delay_main": 300},
    {"test_delay_side": 300, "fix_all": 1}, {"fix_all": 1}, {"fix_all": 1, "sim_hiprio": 0},
    {"edge_stream": 0}, {"sl_phi": 0}, {"sl_phi": 0, "fused_fluid": 0},
    {"edge_stream": 0, "sl_phi": 0, "test_delay_side": 300}, {"skip_marked_rows": 0},
    {"tail_stream": 0}, {"tail_stream": 1, "test_delay_side": 300}, {"diag_first": 1},
    {"fused_fixprep": 0, "diag_first": 1}, {"sl_zero_flags": 0},
], ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_schedule_switch_is_bit_identical(default_run, opts):
    _same(_run(opts), default_run)


@pytest.mark.parametrize("opts", [None, {"fused_fixprep": 0}], ids=["fixprep", "no_fixprep"])
def test_forced_fallback_sweep_is_bit_identical(default_run, opts):
    _same(_run(opts, ex_mode=2), default_run)


def test_diag_seg_switch(default_run):
    got = _run({"diag_seg": 0})
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], default_run[f], err_msg=f)
    for k in ("d_minJ", "d_maxJ", "d_dt", "d_t"):
        np.testing.assert_array_equal(got[k], default_run[k], err_msg=k)
    for k in ("d_cx", "d_cy"):
        np.testing.assert_allclose(got[k], default_run[k], rtol=1e-14, err_msg=k)


def test_option_names_and_errors(gpu):
    from pyrmt_amd import functions as F
    c = F._Ctx(64, 64, 0)
    assert c.get_option("chain_cols") in (1, 2, 3, 4, 5, 6, 7, 8)
    c.set_option("chain_layer_groups", 2)
    assert c.get_option("chain_layer_groups") == 2
    with pytest.raises(Exception, match="unknown option"):
        c.set_option("no_such_switch", 1)


CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
from pyrmt_amd.simulation import soft_disc_in_lid_driven
s = soft_disc_in_lid_driven(256)
assert s.ctx.get_option("chain_layer_groups") == 1 and s.ctx.get_option("fix_all") == 1
s.step(12)
np.savez(sys.argv[2], **{f: s.get(f) for f in %r})
""" % (FIELDS,)


def test_environment_sets_context_defaults(tmp_path, default_run):
    out = str(tmp_path / "env.npz")
    env = dict(os.environ, RMT_CH_LAYERS="1", RMT_FIX_ALL="1")
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, out], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    got = np.load(out)
    for f in FIELDS:
        np.testing.assert_array_equal(got[f], default_run[f], err_msg=f)


def _split_run(options, edit):
    """Three calls of 4 steps; between the first two the map is edited from outside (a +0.0
    tile of X1 set to 1e-300, then back to +0.0 after the second), so the zero-tile flags must
    be rebuilt at every call."""
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    s = soft_disc_in_lid_driven(256, options=options)
    s.step(4)
    if edit:
        x = s.get("X1"); x[2:6, 2:66] = 1e-300; s.set_field("X1", x); s.invalidate()
    s.step(4)
    if edit:
        x = s.get("X1"); x[2:6, 2:66] = 0.0; s.set_field("X1", x); s.invalidate()
    s.step(4)
    out = {f: s.get(f) for f in FIELDS}
    out.update({"d_" + k: np.asarray(v) for k, v in s.diagnostics().items()})
    return out


@pytest.mark.parametrize("edit", [False, True], ids=["plain", "edited"])
def test_sl_zero_flags_across_calls(gpu, edit):
    """The zero-tile flags (sl_zero_flags) are valid only for maps the call itself wrote: split
    calls, with and without an outside edit of the map in between, give the bits of the pass
    without them."""
    _same(_split_run(None, edit), _split_run({"sl_zero_flags": 0}, edit))
