"""Relative error of the GPU DCT Poisson solve against scipy's pocketfft (the reference's own
call, functions.py:1107-1119) per grid shape, under the current RMT_* environment:
python tools/dct_err.py [ny,nx ...].  A measurement aid for DCT variants (test_dct_solve_sizes
holds the bar)."""
import sys

import numpy as np
from scipy.fft import dctn, idctn

import pyrmt_amd


def main():
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or \
        [(49, 49), (257, 129), (300, 4096), (1024, 1024), (4096, 4096), (30, 94)]
    for ny, nx in shapes:
        dx, dy = 1.0 / (nx - 1), 1.0 / (ny - 1)
        rng = np.random.default_rng(ny * 7 + nx)
        rhs = rng.standard_normal((ny, nx))
        eig = pyrmt_amd._precompute_poisson_eigenvalues(nx, ny, dx, dy)
        ref = idctn(dctn(rhs, type=1) / eig, type=1)
        ref -= ref.mean()
        got = pyrmt_amd._solve_poisson_dct(rhs, eig)
        print(f"{ny}x{nx}: {np.abs(got - ref).max() / np.abs(ref).max():.3e}", flush=True)


if __name__ == "__main__":
    main()
