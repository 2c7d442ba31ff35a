"""Repo-root shim for the reference ``physics`` module (drop-in, see sitecustomize.py).

The reference module holds more than the divergence: ``clean_divergence`` (main.py:10),
``solve_poisson`` (velocity_analysis.py:298), the sparse operators and cleaning solvers
(physics.py:55-514), which stay on the host.  When the reference ``physics.py`` is on the
path (next to the caller's script), it is loaded under a private name and every one of its
names is re-exported; only ``compute_consistent_divergence`` (physics.py:6-53) is replaced
by the MI355X kernel, also inside the reference module, so that the cleaning loops
(physics.py:173, :193-194) call the GPU stencil too (bit-identical results).  Without the
reference module (the GPU box), only the divergence is provided.
"""
import importlib.util as _ilu
import os as _os
import sys as _sys

from ptv_interpolation_amd.physics import compute_consistent_divergence as _gpu_divergence

compute_consistent_divergence = _gpu_divergence

_ROOT = _os.path.dirname(_os.path.abspath(__file__))


def _reference_module():
    key = "_ptv_reference_physics"
    if key in _sys.modules:
        return _sys.modules[key]
    for d in _sys.path:
        d = _os.path.abspath(d or _os.getcwd())
        f = _os.path.join(d, "physics.py")
        if d == _ROOT or not _os.path.isfile(f):
            continue
        spec = _ilu.spec_from_file_location(key, f)
        mod = _ilu.module_from_spec(spec)
        _sys.modules[key] = mod
        try:
            spec.loader.exec_module(mod)
        except BaseException:
            del _sys.modules[key]
            raise
        return mod
    return None


_ref = _reference_module()
if _ref is not None:
    globals().update({k: v for k, v in vars(_ref).items() if not k.startswith("__")})
    _ref.compute_consistent_divergence = _gpu_divergence
    compute_consistent_divergence = _gpu_divergence
