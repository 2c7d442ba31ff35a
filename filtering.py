"""Repo-root shim: with this repo first on ``PYTHONPATH`` the reference ``main.py``
(``from filtering import apply_filters``, main.py:12,19) imports the MI355X filter."""
from ptv_interpolation_amd.filtering import *  # noqa: F401,F403
