"""The zero-edit drop-in (sitecustomize.py + the repo-root shims): the reference ``main.py``
imports the MI355X modules when this repo is on ``PYTHONPATH``, and the ``physics`` shim
keeps every reference name (``clean_divergence``, ``solve_poisson``, ...).

CPU only, runs where the reference checkout exists (this container); the reference never
travels to the GPU box, so there it skips.  ``tifffile`` (absent from this image) is
stubbed in a temporary directory for the import.
"""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

pytestmark = pytest.mark.skipif(not os.path.isfile(os.path.join(REF, "main.py")),
                                reason="reference checkout not present (GPU box)")


def _run(code, tmp_path, extra_env=None):
    stub = tmp_path / "stub"
    stub.mkdir(exist_ok=True)
    (stub / "tifffile.py").write_text("def imread(*a, **k):\n    raise OSError('stub')\n"
                                      "def imwrite(*a, **k):\n    raise OSError('stub')\n")
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([ROOT, str(stub)])
    env["MPLBACKEND"] = "Agg"
    env.update(extra_env or {})
    script = tmp_path / "probe.py"
    script.write_text(textwrap.dedent(code))
    # run the probe as a script in the reference directory: its own directory comes first
    # on sys.path, exactly like `python main.py` there
    r = subprocess.run([sys.executable, "-c", f"import runpy, sys; sys.path.insert(0, {REF!r}); "
                        f"runpy.run_path({str(script)!r}, run_name='__main__')"],
                       cwd=REF, env=env, capture_output=True, text=True, timeout=240)
    return r


def test_main_imports_the_mi355x_modules(tmp_path):
    r = _run("""
        import main
        import interpolator, filtering, physics
        assert main.interpolate_field.__module__ == "ptv_interpolation_amd.interpolator", main.interpolate_field.__module__
        assert main.apply_filters.__module__ == "ptv_interpolation_amd.filtering"
        assert main.load_ptv_data.__module__ == "ptv_interpolation_amd.interpolator"
        # physics: the reference names survive, the divergence is the GPU one everywhere
        assert callable(main.clean_divergence) and callable(physics.solve_poisson)
        assert physics.compute_consistent_divergence.__module__ == "ptv_interpolation_amd.physics"
        ref = __import__("sys").modules["_ptv_reference_physics"]
        assert ref.compute_consistent_divergence is physics.compute_consistent_divergence
        import velocity_analysis  # velocity_analysis.py:298 imports solve_poisson lazily
        from physics import solve_poisson, build_laplacian_matrix, clean_divergence_variational
        print("ok")
    """, tmp_path)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().endswith("ok")


def test_dropin_can_be_disabled(tmp_path):
    r = _run("""
        import main
        assert main.interpolate_field.__module__ == "interpolator", main.interpolate_field.__module__
        print("ok")
    """, tmp_path, {"PTV_DROPIN": "0"})
    assert r.returncode == 0, r.stdout + r.stderr
