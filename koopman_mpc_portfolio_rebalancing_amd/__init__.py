"""MI355X-native Koopman-MPC window engine (drop-in for the reference's mpc/backtest hot path)."""
from .mpc import MPCConfig, solve_mpc_log_utility, solve_mpc_log_utility_batched  # noqa: F401

__version__ = "0.1.0"
