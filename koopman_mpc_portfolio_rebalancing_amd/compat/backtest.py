"""``backtest`` shim: the reference module's names (backtest.py:22-249) on the gfx950 window path."""
from koopman_mpc_portfolio_rebalancing_amd.backtest import (BacktestConfig, BuyAndHoldStrategy,  # noqa: F401
                                                            KoopmanMPCStrategy, Strategy,
                                                            calculate_metrics, run_backtest)
from koopman_mpc_portfolio_rebalancing_amd.mpc import MPCConfig, solve_mpc_log_utility  # noqa: F401
