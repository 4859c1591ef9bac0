"""pyrmt_amd -- MI355X-native 2D Reference Map Technique (RMT) time step.

Drop-in for pyRMT's per-step hot path (pyRMT/__init__.py:1-57 operator surface): the
operators run as hand-written HIP kernels for gfx950 in librmt.so (include/rmt.h), with
a device-resident fused step (pyrmt_amd.simulation) for the benchmark loop bodies.
"""
from . import _lib
from .bc import NoSlipLid, FreeSlipBox, Periodic, Disc
from .functions import *  # noqa: F401,F403  (the reference's operator names)
from .functions import (_precompute_poisson_eigenvalues, _solve_poisson_dct,  # noqa: F401
                        _compute_divergence_rc, _compute_divergence, _compute_pressure_gradient,
                        _weno5_rhs, _precompute_poisson_eigenvalues_periodic,
                        _tile_overlap, _solve_poisson_fft, _compute_divergence_periodic,
                        _compute_pressure_gradient_periodic, _central2_rhs,
                        _conservative_rhs)
from .output import output_simulation_data  # noqa: F401  (pyRMT/__init__.py:32)
from . import simulation
from . import mac

__version__ = "0.1.0"


def library():
    """The loaded librmt.so (raises ImportError if it was not built)."""
    return _lib.lib()
