"""The fused step's schedule switches (read once per process, so each runs in its own child
process) against the default schedule: every one reorders or overlaps the same kernels, so
fields and diagnostics must be bit-identical.  N=256 so that the split
projection (LDS DCT plan: 255 = 3 5 17) and with it the early transpose are on.

  RMT_SIM_HIPRIO=0        the step on the caller's stream instead of the highest-priority one
  RMT_EARLY_TRANSPOSE=0   the column pass's transpose entirely after the chain
  RMT_EARLY_GEOMETRY=0    the next step's extrapolation geometry on the main stream
  RMT_SIDE_TAIL=0         p -= mean(p) and the diagnostics right after the projection
  RMT_NO_OVERLAP=1        no second stream at all
  RMT_SIM_SYNC=1          dt read back on the host every step
  RMT_CH_PARTS=1          the chain in one workgroup
  RMT_CH_PARTS=4          the chain in four column parts (more cross-part hand-offs)
  RMT_FUSED_FLUID=0       the momentum's pure-fluid flags from their own pass over phi
  TEST_EX_MODE=2          (this file's child) the extrapolation's forced fallback sweep, which
                          the fused step runs on its second stream beside the chain
  RMT_FUSED_FIXPREP=0     the fix-up's phi and momentum prep in two kernels (the sweep in order)
  RMT_EXT_EVENTS=0        the cross-stream events recorded after their kernels instead of
                          completing with them (hipExtLaunchKernel)
  RMT_MERGED_JOIN=0       the second stream joined twice (after its momentum, before the
                          projection) instead of once after its row passes
  RMT_TEST_DELAY_SIDE=300 the second stream sleeps ~1 ms as its work beside the chain starts
  RMT_TEST_DELAY_MAIN=300 the critical stream sleeps ~1 ms right after the chain (both: every
                          cross-stream read is ordered by an event, whatever the timing)
  RMT_FIX_ALL=1           the fix-up re-runs phi, the prep and the four stages on EVERY tile
                          (interior, edge and domain-boundary tiles through the list kernels;
                          the default's fix-up list holds interior tiles only for this disc) --
                          the regression test for the round-3 divergent list-kernel variant
                          
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("u", "v", "p", "X1", "X2", "phi", "J")
CHILD = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import os
from pyrmt_amd.simulation import soft_disc_in_lid_driven
from pyrmt_amd.functions import extrapolation_mode
if os.environ.get("TEST_EX_MODE"):
    extrapolation_mode(int(os.environ["TEST_EX_MODE"]))
s = soft_disc_in_lid_driven(256)
s.step(12)
out = {f: s.get(f) for f in %r}
out.update({"d_" + k: np.asarray(v) for k, v in s.diagnostics().items()})
np.savez(sys.argv[2], **out)
""" % (FIELDS,)


def _run(tmp_path, tag, env_extra):
    out = str(tmp_path / f"{tag}.npz")
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, out], env=env, capture_output=True,
                       text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(out)


@pytest.fixture(scope="module")
def default_run(tmp_path_factory, gpu):
    return _run(tmp_path_factory.mktemp("env"), "default", {})


@pytest.mark.parametrize("env", [
    {"RMT_SIM_HIPRIO": "0"}, {"RMT_EARLY_TRANSPOSE": "0"}, {"RMT_EARLY_GEOMETRY": "0"},
    {"RMT_SIDE_TAIL": "0"}, {"RMT_NO_OVERLAP": "1"}, {"RMT_SIM_SYNC": "1"},
    {"RMT_CH_PARTS": "1"}, {"RMT_CH_PARTS": "4"}, {"RMT_FUSED_FLUID": "0"},
    {"TEST_EX_MODE": "2"}, {"TEST_EX_MODE": "2", "RMT_FUSED_FIXPREP": "0"},
    {"RMT_FUSED_FIXPREP": "0"}, {"RMT_EXT_EVENTS": "0"},
    {"RMT_MERGED_JOIN": "0"}, {"RMT_TEST_DELAY_SIDE": "300"}, {"RMT_TEST_DELAY_MAIN": "300"},
    {"RMT_TEST_DELAY_SIDE": "300", "RMT_FIX_ALL": "1"}, {"RMT_FIX_ALL": "1"}, {"RMT_FIX_ALL": "1", "RMT_SIM_HIPRIO": "0"},
], ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_schedule_switch_is_bit_identical(tmp_path, default_run, env):
    got = _run(tmp_path, "variant", env)
    assert sorted(got.files) == sorted(default_run.files)
    for k in default_run.files:
        np.testing.assert_array_equal(got[k], default_run[k], err_msg=k)
