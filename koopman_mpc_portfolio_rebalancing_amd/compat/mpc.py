"""``mpc`` shim: the reference module's names (mpc.py:17-184) on the gfx950 solve kernels."""
from koopman_mpc_portfolio_rebalancing_amd.mpc import (MPCConfig, solve_mpc_log_utility,  # noqa: F401
                                                       solve_mpc_log_utility_batched,
                                                       solve_mpc_mean_variance,
                                                       solve_mpc_mean_variance_batched)
