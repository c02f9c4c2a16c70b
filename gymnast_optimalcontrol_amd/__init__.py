"""gymnast_optimalcontrol_amd -- MI355X-native batched acrobot Newton/Armijo swing-up optimiser.

Drop-in for the hot path of francescoolivieri/Gymnast_OptimalControl: the call surface of its
``dynamics.py`` and ``trajectory_generation.py`` (modules of the same names here), computed by
hand-written gfx950 HIP kernels behind the C-ABI of include/gymnast_acrobot.h.

Heavy imports (torch, the HIP library) happen lazily when a submodule is used.
"""
__version__ = "0.1.0"

__all__ = ["dynamics", "trajectory_generation", "engine", "solver", "distributed", "params"]
