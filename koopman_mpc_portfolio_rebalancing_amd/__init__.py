"""MI355X-native Koopman-MPC window engine.

Drop-in for the reference's per-window hot path (yli421/koopman-mpc-portfolio-rebalancing):
``MPCConfig`` / ``solve_mpc_log_utility`` (mpc.py) and ``BacktestConfig`` / ``Strategy`` /
``BuyAndHoldStrategy`` / ``KoopmanMPCStrategy`` / ``run_backtest`` / ``calculate_metrics``
(backtest.py), executed by hand-written gfx950 kernels in libkmpc.so (C ABI: include/kmpc.h).
"""
from .mpc import (MPCConfig, gross_returns, log_utility_value_batched, solve_mpc_log_utility,  # noqa: F401
                  solve_mpc_log_utility_batched, solve_mpc_mean_variance, solve_mpc_mean_variance_batched)
from .koopman import DeviceKoopman, KoopmanModelSpec, standardize_panel  # noqa: F401
from .backtest import (BacktestConfig, BuyAndHoldStrategy, KoopmanMPCStrategy, Strategy,  # noqa: F401
                       calculate_metrics, run_backtest, run_backtest_lockstep)

__version__ = "0.6.0"
