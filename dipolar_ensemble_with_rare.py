"""Import shim: lets the reference's unmodified ``sweep_sea_detuning.py`` (which does
``from dipolar_ensemble_with_rare import ...``, sweep_sea_detuning.py:103-109) run on the
MI355X engine when this repository root is on ``sys.path``."""
from quantumsimulations_amd.dipolar_ensemble_with_rare import *  # noqa: F401,F403
from quantumsimulations_amd.dipolar_ensemble_with_rare import (  # noqa: F401
    DipolarRareParams,
    build_hamiltonian_rare,
    dipolar_couplings_from_positions,
    dims_with_rare,
    get_derived_frequencies,
    initial_state_rare,
    shell_positions_with_rare_center,
    simulate_rare,
    simulate_rare_batch,
)
