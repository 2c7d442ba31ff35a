"""Golden end-to-end fixtures of the reference ``main.py`` pipeline (main.py:21-246) on C1.

Runs the reference ``main.py`` itself, as a subprocess, on the BASELINE C1 case (a 10k
sphere-pack particle CSV in voxel units): an unmasked IDW run and a masked run with the
pore-mask path (sample_mask_on_grid, extract_boundary_particles), the outlier filter and the
NaN-fill / mask epilogue.  Commits the inputs (the CSV text, the raw mask, the arguments),
the NPZ arrays main.py writes (main.py:220-226) and its stdout.  ``tests/test_gpu_main_pipeline.py``
replays the same steps through the drop-in modules on the GPU and compares.

Runs only where the read-only reference checkout exists.  ``tifffile`` is absent from this
image: a stub module whose ``imread(path)`` returns ``numpy.load(path + ".npy")`` stands in
for the mask TIFF reader (interpolator.py:35); no TIFF is written (no --output-tif).

Usage:  python tests/golden/make_main_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

RUNS = {
    # name: (main.py arguments, masked)
    "main_c1_idw": (["--method", "idw", "--idw-neighbors", "8"], False),
    "main_c1_masked": (["--method", "idw", "--idw-neighbors", "8", "--downscale", "2", "--boundary-particles",
                        "--boundary-sampling", "3", "--filter-outliers"], True),
}


def _inputs():
    sys.path.insert(0, ROOT)
    from ptv_interpolation_amd import synth

    G = 64
    P, _ = synth.sphere_pack(10_000, G, seed=77)
    rng = np.random.default_rng(78)
    u = np.sin(P[:, 0] / 9.0) + 0.05 * rng.standard_normal(len(P))
    v = np.cos(P[:, 1] / 7.0) + 0.05 * rng.standard_normal(len(P))
    w = 1.0 + 0.1 * np.sin(P[:, 2] / 5.0) + 0.05 * rng.standard_normal(len(P))
    Q = np.stack([u, v, w], 1)
    bad = rng.choice(len(P), 150, replace=False)
    Q[bad] *= rng.uniform(3.0, 20.0, (150, 1))  # MAD outliers, some above --filter-max-speed 10
    import pandas as pd

    df = pd.DataFrame({"x": P[:, 0], "y": P[:, 1], "z": P[:, 2], "vx": Q[:, 0], "vy": Q[:, 1], "vz": Q[:, 2]})
    csv = df.to_csv(index=False)
    fluid = synth.fluid_mask(G)
    return csv, fluid


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    a = ap.parse_args()
    csv, fluid = _inputs()
    with tempfile.TemporaryDirectory() as td:
        stub = os.path.join(td, "stub")
        os.makedirs(stub)
        with open(os.path.join(stub, "tifffile.py"), "w") as f:
            f.write("import numpy as np\n\ndef imread(path, *a, **k):\n    return np.load(path + '.npy')\n\n"
                    "def imwrite(*a, **k):\n    raise OSError('stub: no TIFF output')\n")
        csv_path = os.path.join(td, "c1.csv")
        with open(csv_path, "w") as f:
            f.write(csv)
        mask_path = os.path.join(td, "mask.tif")
        np.save(mask_path + ".npy", fluid.astype(np.uint8))  # load_mask: > 0 is fluid (interpolator.py:37)
        env = dict(os.environ, PYTHONPATH=stub, MPLBACKEND="Agg", PTV_DROPIN="0")
        for name, (args, masked) in RUNS.items():
            out = os.path.join(td, name + ".npz")
            cmd = [sys.executable, os.path.join(a.ref, "main.py"), "--input", csv_path, "--no-plot",
                   "--output-npz", out] + (["--mask", mask_path] if masked else []) + args
            r = subprocess.run(cmd, cwd=td, env=env, capture_output=True, text=True, timeout=600)
            if r.returncode != 0:
                raise RuntimeError(r.stdout + r.stderr)
            with np.load(out, allow_pickle=False) as z:
                res = {f"out_{k}": z[k] for k in z.files}
            import scipy

            np.savez_compressed(os.path.join(HERE, name + ".npz"), csv=np.array(csv), args=np.array(args),
                                masked=int(masked), mask_raw=fluid if masked else np.zeros(0, bool),
                                stdout=np.array(r.stdout.replace(td, "<tmp>")), numpy_version=np.array(np.__version__),
                                scipy_version=np.array(scipy.__version__), **res)
            print("wrote", name, {k: v.shape for k, v in res.items()})


if __name__ == "__main__":
    main()
