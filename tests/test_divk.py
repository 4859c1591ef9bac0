"""divk (pyrmt_amd/csrc/divk.hpp): the correctly rounded division by a precomputed divisor
that the stencil kernels use in place of x / (2h), x / (6h), xq / dx, x / (rho + 1e-12).
It must equal IEEE division bit for bit, or every "bit-exact" bar downstream is void.

  * CPU: tools/divk_check.hip (host code, the same header) against x / d on the hardest
    operands -- x / d within ~2^-105 relative of a rounding midpoint, from Dint^-1 mod 2^54
    -- plus random and special operands, for the divisors of every config grid.
  * GPU: the device code (rmt_selftest_divk) against x / d on the device and in numpy, on
    hard operands built here with Python integers.
"""
import os
import random
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def test_divk_host_check(tmp_path):
    exe = str(tmp_path / "divk_check")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O2", "-std=c++17", "-ffp-contract=off", "-o", exe,
                    os.path.join(ROOT, "tools", "divk_check.hip")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "OK: divk == IEEE division on every operand" in r.stdout
    # the generator reaches operands next to a midpoint: x * RN(1/d) misrounds on them
    assert "x*RN(1/d) on 0 of them" not in r.stdout.splitlines()[3]


def hard_operands(d, count=4000, seed=1):
    """x (float64) with x / d within ~2^-105 relative of a midpoint of the quotient's binade:
    M * Dint = X * 2^s + k (M odd, small k), x = X * 2^(s - 105), scaled by powers of 2."""
    m, e = np.frexp(d)
    dint = int(np.ldexp(m, 53))           # 53-bit integer significand
    tz = (dint & -dint).bit_length() - 1
    dodd = dint >> tz
    rng = random.Random(seed)
    out = []
    k = 1
    while len(out) < count and k < 20001:
        for ko in (k, -k):
            kk = ko << tz
            for s in (53, 54):
                sm = s - tz
                if sm < 40:          # d = 2^e (and nearby): every quotient is exact
                    continue
                M = (ko * pow(dodd, -1, 1 << sm)) % (1 << sm)
                if M <= (1 << 53):
                    M += (((1 << 53) - M) // (1 << sm) + 1) << sm
                if M >= (1 << 54) or not (M & 1):
                    continue
                P = M * dint - kk
                if P % (1 << s):
                    continue
                X = P >> s
                if not ((1 << 52) <= X < (1 << 53)):
                    continue
                x = float(np.ldexp(float(X), s - 105))
                sc = rng.randrange(-850, 950)
                out.append(float(np.ldexp(x, sc)) * (1 if rng.random() < 0.5 else -1))
        k += 2
    return np.array(out, dtype=np.float64)


DIVISORS = [2.0 / 4095, 6.0 / 4095, 1.0 / 4095, 2.0 / 255, 6.0 / 255, 2.0 / 1023,
            6.0 / 1023, 1.0 + 1e-12, 2.0 / 64, 1.0 / 8191, 0.7, 1.9999999999999,
            3.0e-9, 7.0e30]   # outside the certified exponents (IEEE division)


def test_hard_operands_generator():
    """CPU: the generator terminates for every divisor of the GPU test and its operands are
    hard (x * RN(1/d) misrounds on a good share of them)."""
    for d in DIVISORS:
        h = hard_operands(d)
        if d == 2.0 / 64:
            assert len(h) == 0
            continue
        assert len(h) >= 1000
        assert (h * np.float64(1.0 / d) != h / d).sum() > len(h) // 10


@pytest.mark.gpu
def test_divk_device_bitwise(gpu):
    import torch
    from pyrmt_amd import _lib as L
    from pyrmt_amd.functions import ctx_for, _p
    rng = np.random.default_rng(7)
    for d in DIVISORS:
        hard = hard_operands(d)
        bits = rng.integers(0, 2 ** 63, size=200000, dtype=np.int64)
        rand = bits.view(np.float64)
        rand = rand[np.isfinite(rand)]
        spec = np.array([0.0, -0.0, 5e-324, -5e-324, 2.2250738585072014e-308, 2.0 ** -900,
                         2.0 ** -901, 2.0 ** 1000, np.inf, -np.inf, np.nan, 1.0, d, -d, 3 * d],
                        dtype=np.float64)
        x = np.concatenate([hard, -rand, rand, spec])
        xt = torch.from_numpy(x).cuda()
        q = torch.empty_like(xt)
        qi = torch.empty_like(xt)
        c = ctx_for(8, 8)
        L.check(L.lib().rmt_selftest_divk(c.bind(), _p(xt), xt.numel(), d, _p(q), _p(qi)),
                "selftest_divk")
        qn, qin = q.cpu().numpy(), qi.cpu().numpy()
        ref = x / d
        same = lambda a, b: (a.view(np.uint64) == b.view(np.uint64)) | (np.isnan(a) & np.isnan(b))
        assert same(qin, ref).all(), f"device IEEE division differs from numpy for d={d!r}"
        bad = ~same(qn, ref)
        assert not bad.any(), (d, x[bad][:5], qn[bad][:5], ref[bad][:5])
