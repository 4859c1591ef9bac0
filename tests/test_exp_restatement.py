"""The device exp used for the extrapolation weights (pyrmt_amd/csrc/exp_glibc.h) must be
bit-identical to the libm exp the reference uses (Numba scalar exp = glibc exp).  The
same header is compiled here for the host and compared on the weight domain [-1, 0]."""
import os
import subprocess
import tempfile

import pytest

from conftest import ROOT

SRC = r'''
#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdint>
#include "exp_glibc.h"
int main() {
    long n = 4000000, bad = 0;
    uint64_t s = 88172645463325252ull;
    for (long k = 0; k < n; ++k) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        double x = -(double)(s >> 11) * 0x1p-53;
        if (k % 4 == 0) x = -(double)((s >> 20) % 81) / 32.0;   // d^2/r^2 of window cells
        if (k == 1) x = -0.0;
        if (k == 2) x = -1e-300;
        double a = rmt::exp_glibc(x), b = std::exp(x);
        uint64_t ua, ub; std::memcpy(&ua, &a, 8); std::memcpy(&ub, &b, 8);
        if (ua != ub) ++bad;
    }
    std::printf("%ld\n", bad);
    return 0;
}
'''


def test_device_exp_matches_libm_bitwise():
    gxx = "g++"
    if subprocess.run(["which", gxx], capture_output=True).returncode:
        pytest.skip("no g++")
    d = tempfile.mkdtemp()
    src = os.path.join(d, "t.cpp")
    open(src, "w").write(SRC)
    exe = os.path.join(d, "t")
    subprocess.run([gxx, "-O2", "-std=c++17", "-ffp-contract=off", "-I",
                    os.path.join(ROOT, "pyrmt_amd", "csrc"), src, "-o", exe], check=True)
    out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout
    assert int(out.strip()) == 0
