"""Bit-compare the local-RBF output of two library builds (dev tool, GPU box).

usage: python tools/rbf_bitcompare.py libA.so libB.so [kernel]
Runs the same Gaussian (or given kernel) case under PTV_LIB=libA and PTV_LIB=libB in
separate processes and reports whether U, V, W are bit-identical."""
import os
import subprocess
import sys
import tempfile

import numpy as np

CASE = r'''
import sys, numpy as np
sys.path.insert(0, %r)
from ptv_interpolation_amd.rbf import LocalRBFInterpolator
rng = np.random.default_rng(5)
P = rng.uniform(0, 31, (20000, 3)); Q = rng.standard_normal((20000, 3))
ax = np.linspace(0, 31, 32)
kern = %r
kw = dict(epsilon=0.3, degree=-1) if kern == "gaussian" else {}
U, V, W = LocalRBFInterpolator(P, Q, neighbors=32, kernel=kern, **kw).evaluate_grid(ax, ax, ax)
np.savez(%r, U=U, V=V, W=W)
'''


def main():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    kern = sys.argv[3] if len(sys.argv) > 3 else "gaussian"
    outs = []
    for lib in sys.argv[1:3]:
        f = tempfile.mktemp(suffix=".npz")
        env = dict(os.environ, PTV_LIB=os.path.realpath(lib))
        subprocess.run([sys.executable, "-c", CASE % (root, kern, f)], env=env, check=True)
        outs.append(np.load(f))
    same = all(np.array_equal(outs[0][c], outs[1][c]) for c in "UVW")
    d = max(float(np.max(np.abs(outs[0][c] - outs[1][c]))) for c in "UVW")
    print(f"{kern}: bit-identical={same} max|d|={d:.3e}")


if __name__ == "__main__":
    main()
