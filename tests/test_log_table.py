"""The null-space RBF kernel's thin-plate-spline log (log_tab in ptv_rbf_ns.hpp): the committed
table is what tools/gen_log_table.py generates, and the reduction it drives (restated here in
numpy, operation for operation) is within 3 ulp of the correctly rounded log over the ranges the
kernel sees, with exact zeros at x = 1."""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "ptv_interpolation_amd", "csrc", "ptv_log_table.hpp")


def _table():
    txt = open(HDR).read()
    pairs = re.findall(r"\{(-?0x[0-9a-fp.+-]+), (-?0x[0-9a-fp.+-]+)\}", txt)
    assert len(pairs) == 512
    return np.array([[float.fromhex(a), float.fromhex(b)] for a, b in pairs])


def test_committed_table_is_generated():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_log_table.py")], capture_output=True,
                         text=True, check=True).stdout
    assert out == open(HDR).read()


def _log_tab(x, tab):
    # frexp: x = m 2^e, m in [1/2, 1); bin = top 9 fraction bits of m (bits 11..19 of the high word)
    m, e = np.frexp(x)
    hi = (m.view(np.uint64) >> np.uint64(32)).astype(np.int64)
    i = (hi >> 11) & 511
    s, t = tab[i, 0], tab[i, 1]
    r = _fma(m, s, -1.0)  # the device's v_fma_f64 (emulated: Dekker two-product + compensated sum)
    ee = np.where(i < 256, e - 1, e).astype(np.float64)
    tt = _fma(ee, float.fromhex("0x1.62e42fefa39efp-1"), t)
    h = _fma(r, -1.0 / 6.0, 0.2)
    h = _fma(r, h, -0.25)
    h = _fma(r, h, 1.0 / 3.0)
    h = _fma(r, h, -0.5)
    return tt + _fma(r * r, h, r)


def _two_prod(a, b):
    p = a * b
    sp = 134217729.0
    ah = a * sp
    ah = ah - (ah - a)
    al = a - ah
    bh = b * sp
    bh = bh - (bh - b)
    bl = b - bh
    return p, ((ah * bh - p) + ah * bl + al * bh) + al * bl


def _fma(a, b, c):
    # correctly rounded to within the double-double sum's error (enough for a 3-ulp bound test)
    a, b, c = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64), np.asarray(c, np.float64))
    p, pe = _two_prod(a, b)
    s = p + c
    bv = s - p
    err = (p - (s - bv)) + (c - bv)
    return s + (err + pe)


def test_log_tab_accuracy():
    tab = _table()
    rng = np.random.default_rng(5)
    xs = np.concatenate([
        np.ldexp(1.0 + rng.random(200_000), rng.integers(-40, 40, 200_000)),  # wide range
        1.0 + (rng.random(100_000) - 0.5) * 2.0 ** -7,                          # around 1
        np.ldexp(1.0 - rng.random(100_000) * 2.0 ** -9, rng.integers(-1, 2, 100_000)),  # just below powers of 2
    ])
    got = _log_tab(xs, tab)
    ref = np.log(xs.astype(np.longdouble))
    nz = ref != 0
    rel = np.abs((got[nz].astype(np.longdouble) - ref[nz]) / ref[nz]) / np.longdouble(2.0 ** -53)
    assert float(rel.max()) <= 3.0, float(rel.max())
    assert _log_tab(np.array([1.0]), tab)[0] == 0.0
    assert np.isfinite(_log_tab(np.array([0.0]), tab)[0])  # phi(0) = 0.5 * 0 * finite
