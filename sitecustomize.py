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


# files that mark a directory as the reference's layout (its entry scripts)
_MARKERS = ("main.py", "run_porous_glass.py", "interpolate_porous_glass.py", "test_parallel.py", "analyze_flow.py")
_NOTED = set()


def _reference_shadows(name):
    """The first other ``name.py`` on sys.path sits next to one of the reference's entry scripts
    (the reference layout).  Any other module of that name is left alone, with a one-time note on
    stderr (it then runs on the CPU; ``PTV_DROPIN=0`` silences it); with none, the normal import
    finds the shim."""
    for d in sys.path:
        d = os.path.abspath(d or os.getcwd())
        if d == _ROOT:
            continue
        f = os.path.join(d, name + ".py")
        if os.path.isfile(f):
            if any(os.path.isfile(os.path.join(d, m)) for m in _MARKERS):
                return True
            if name not in _NOTED:
                _NOTED.add(name)
                print(f"ptv_interpolation_amd drop-in: {f} is not next to a reference entry script "
                      f"({', '.join(_MARKERS)}); importing it unchanged (CPU). PTV_DROPIN=0 silences this.",
                      file=sys.stderr)
            return False
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
