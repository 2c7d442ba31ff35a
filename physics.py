"""Repo-root shim: with this repo first on ``PYTHONPATH``, ``from physics import
compute_consistent_divergence`` (view_divergence.py:5) resolves to the MI355X kernel."""
from ptv_interpolation_amd.physics import *  # noqa: F401,F403
