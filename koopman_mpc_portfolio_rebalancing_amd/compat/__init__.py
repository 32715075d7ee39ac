"""Drop-in module shims for the reference's flat import layout.

The reference imports its hot-path modules by bare name (``from mpc import ...``,
``from backtest import ...``; reference backtest.py:18, baselines.py:20-21, run_experiment.py:23,
tests/test_mpc.py:4, tests/test_backtest.py:7). Putting this directory first on ``sys.path``
(``sys.path.insert(0, koopman_mpc_portfolio_rebalancing_amd.compat.PATH)``) makes those imports
resolve to the gfx950 engine; everything else in the reference (config, model, data_finance) is
untouched. See INTEGRATION.md.
"""
import os

PATH = os.path.dirname(os.path.abspath(__file__))
