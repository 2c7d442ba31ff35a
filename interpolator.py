"""Repo-root shim: ``PYTHONPATH=/path/to/this/repo python main.py ...`` makes the
reference drivers (main.py, test_parallel.py, run_porous_glass.py) import the
MI355X implementation in place of the reference ``interpolator.py``."""
from ptv_interpolation_amd.interpolator import *  # noqa: F401,F403
from ptv_interpolation_amd.interpolator import separable_axes  # noqa: F401
