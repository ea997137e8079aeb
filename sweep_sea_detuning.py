"""Import shim: ``import sweep_sea_detuning`` from this repository root gives the MI355X
batched sweep with the reference module's public names (quantumsimulations_amd/sweep_sea_detuning.py)."""
from quantumsimulations_amd.sweep_sea_detuning import *  # noqa: F401,F403
from quantumsimulations_amd.sweep_sea_detuning import (  # noqa: F401
    SLOPE_T_MIN,
    _safe_normalized_difference,
    coarse_grain,
    contrast_michelson_with_t_gate,
    detuning_label,
    f1R_for_resonance,
    iz_slope_from_coarse,
    main,
    run_sweep_sea_detuning,
)

if __name__ == "__main__":
    main()
