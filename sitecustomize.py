"""Zero-edit drop-in hook for the reference scripts.

``PYTHONPATH=/path/to/this/repo python main.py ...`` run from the reference directory puts the
script's own directory ahead of ``PYTHONPATH`` on ``sys.path``, so a plain module on the path
can never shadow the reference ``interpolator.py`` / ``filtering.py`` / ``physics.py`` that sit
next to ``main.py``.  Python imports ``sitecustomize`` from ``PYTHONPATH`` at start-up, before
the script directory is added; this one installs a meta-path finder that resolves those three
top-level module names to the repo-root shims (``interpolator.py``, ``filtering.py``,
``physics.py``), which re-export the MI355X implementations.  Child processes inherit
``PYTHONPATH``, so ``run_porous_glass.py``'s ``subprocess.run(["python", "main.py", ...])``
(run_porous_glass.py:37-59) picks the drop-in up too.  ``PTV_DROPIN=0`` turns it off.

The system's own ``sitecustomize`` (the next one on the path) is still executed.
"""
import importlib.abc
import importlib.util
import os
import sys

_ROOT = os.path.dirname(os.path.abspath(__file__))
_SHADOWED = ("interpolator", "filtering", "physics")


def _reference_shadows(name):
    """The first other ``name.py`` on sys.path sits next to a ``main.py`` (the reference layout).
    Any other module of that name is left alone; with none, the normal import finds the shim."""
    for d in sys.path:
        d = os.path.abspath(d or os.getcwd())
        if d == _ROOT:
            continue
        if os.path.isfile(os.path.join(d, name + ".py")):
            return os.path.isfile(os.path.join(d, "main.py"))
    return False


class _DropInFinder(importlib.abc.MetaPathFinder):
    def find_spec(self, name, path=None, target=None):
        if path is not None or name not in _SHADOWED or os.environ.get("PTV_DROPIN", "1") == "0":
            return None
        if not _reference_shadows(name):
            return None
        return importlib.util.spec_from_file_location(name, os.path.join(_ROOT, name + ".py"))


if not any(isinstance(f, _DropInFinder) for f in sys.meta_path):
    sys.meta_path.insert(0, _DropInFinder())


def _chain_next_sitecustomize():
    for d in sys.path:
        d = os.path.abspath(d or os.getcwd())
        if d == _ROOT:
            continue
        f = os.path.join(d, "sitecustomize.py")
        if os.path.isfile(f):
            spec = importlib.util.spec_from_file_location("_ptv_next_sitecustomize", f)
            mod = importlib.util.module_from_spec(spec)
            try:
                spec.loader.exec_module(mod)
            except Exception as e:  # reported like site.py does, without breaking start-up
                print(f"Error in sitecustomize {f}; set PYTHONVERBOSE for traceback:\n"
                      f"{type(e).__name__}: {e}", file=sys.stderr)
            return


_chain_next_sitecustomize()
