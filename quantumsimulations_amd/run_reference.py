"""Run one of the reference's own scripts UNMODIFIED with this engine as its solver.

    python -m quantumsimulations_amd.run_reference /path/to/reference/sweep_sea_detuning.py [args]

Python puts a script's own directory first on ``sys.path``, so ``python
/path/to/reference/sweep_sea_detuning.py`` would import the reference's sibling
``dipolar_ensemble_with_rare.py`` (and fail on its ``import qutip``,
dipolar_ensemble_with_rare.py:8) even with this repository on PYTHONPATH.  This launcher instead
puts this repository's root first -- whose ``dipolar_ensemble_with_rare.py`` is the MI355X drop-in
(same names, signatures and return contract, sweep_sea_detuning.py:103-109) -- and executes the
script as ``__main__`` without adding the script's directory.
"""
from __future__ import annotations

import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(argv=None) -> None:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv:
        raise SystemExit("usage: python -m quantumsimulations_amd.run_reference SCRIPT [args...]")
    script = os.path.abspath(argv[0])
    sys.path[:] = [ROOT] + [p for p in sys.path if os.path.abspath(p or ".") != os.path.dirname(script)]
    for name in ("dipolar_ensemble_with_rare",):   # a previously imported reference copy
        sys.modules.pop(name, None)
    sys.argv = [script] + argv[1:]
    runpy.run_path(script, run_name="__main__")


if __name__ == "__main__":
    main()
