"""``baselines`` shim: MarkowitzStrategy (baselines.py:24-106) and DMDStrategy (baselines.py:127-187)
on the device kernels."""
from koopman_mpc_portfolio_rebalancing_amd.backtest import Strategy  # noqa: F401
from koopman_mpc_portfolio_rebalancing_amd.baselines import DMDStrategy, MarkowitzStrategy  # noqa: F401
from koopman_mpc_portfolio_rebalancing_amd.mpc import (MPCConfig, solve_mpc_log_utility,  # noqa: F401
                                                       solve_mpc_mean_variance)
