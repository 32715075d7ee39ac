"""``mpc`` shim: the reference module's names (mpc.py:17-117) on the gfx950 solve kernel."""
from koopman_mpc_portfolio_rebalancing_amd.mpc import (MPCConfig, solve_mpc_log_utility,  # noqa: F401
                                                       solve_mpc_log_utility_batched)


def solve_mpc_mean_variance(*args, **kwargs):
    """mpc.py:119-184 (mean-variance QP) is SURVEY §8(f) row 3, not yet on the device."""
    raise NotImplementedError("solve_mpc_mean_variance is not part of the device hot path yet "
                              "(SURVEY.md §8f row 3)")
