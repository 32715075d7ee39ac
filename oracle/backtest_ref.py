"""Plain numpy restatement of the reference backtest loop and metrics — TEST INFRASTRUCTURE ONLY.

run_backtest   follows backtest.py:133-219 (n_steps, initial 1/N weights, cost, realized return,
               value update, drift with the 1e-8 denominator guard, history rows).
calculate_metrics follows backtest.py:221-249 (population std, sqrt(252) Sharpe, drawdown,
               total return relative to the first row).
"""
from __future__ import annotations

import numpy as np


def run_backtest(rebalance, all_returns, n_test, horizon, n_assets, initial_capital=10000.0,
                 rebalance_freq=1, cost_coeff=0.001):
    """rebalance(t, current_weights) -> target weights; all_returns [n_rows, N] de-standardized
    log-returns (backtest.py:169-171). Returns a list of history dicts (without dates)."""
    n_steps = n_test - horizon                                   # backtest.py:150
    portfolio_value = float(initial_capital)
    current_weights = np.ones(n_assets) / n_assets               # backtest.py:161
    history = []
    for t in range(0, n_steps, rebalance_freq):                  # backtest.py:163-173
        target_weights = rebalance(t, current_weights)
        turnover = np.sum(np.abs(target_weights - current_weights))
        cost = cost_coeff * turnover * portfolio_value
        current_weights = target_weights
        portfolio_value -= cost
        port_ret = 0.0
        if t + 1 < len(all_returns):                             # backtest.py:191
            realized_ret = np.exp(all_returns[t + 1]) - 1.0
            port_ret = np.sum(current_weights * realized_ret)
            portfolio_value *= (1.0 + port_ret)
            denom = 1.0 + port_ret
            if abs(denom) < 1e-8:
                denom = 1e-8
            current_weights = current_weights * (1.0 + realized_ret) / denom
        history.append({"portfolio_value": portfolio_value, "return": port_ret,
                        "turnover": turnover, "cost": cost})
    return history


def calculate_metrics(returns, turnover, portfolio_value):
    if len(returns) == 0:
        return {}
    returns = np.asarray(returns)
    mean_ret = np.mean(returns)
    std_ret = np.std(returns)
    sharpe = np.sqrt(252) * mean_ret / (std_ret + 1e-8)
    cum = (1 + returns).cumprod()
    peak = np.maximum.accumulate(cum)
    max_dd = np.min((cum - peak) / peak)
    return {"Sharpe Ratio": sharpe, "Max Drawdown": max_dd, "Avg Turnover": float(np.mean(turnover)),
            "Final Value": portfolio_value[-1],
            "Total Return": portfolio_value[-1] / portfolio_value[0] - 1.0}
