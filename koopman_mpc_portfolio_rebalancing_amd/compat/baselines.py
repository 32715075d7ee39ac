"""``baselines`` shim: DMDStrategy (baselines.py:127-187) on the device window path."""
from koopman_mpc_portfolio_rebalancing_amd.backtest import Strategy  # noqa: F401
from koopman_mpc_portfolio_rebalancing_amd.baselines import DMDStrategy  # noqa: F401
from koopman_mpc_portfolio_rebalancing_amd.mpc import MPCConfig, solve_mpc_log_utility  # noqa: F401


class MarkowitzStrategy(Strategy):
    """baselines.py:23-112 (mean-variance QP) is SURVEY §8(f) row 3 — not on the device yet."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("MarkowitzStrategy (mean-variance QP) is not part of the device path yet "
                                  "(SURVEY.md §8f row 3)")

    def rebalance(self, t, current_weights, env, lookback_window=60):
        raise NotImplementedError
