"""Optimality of the MPC goldens certified without the interior-point iteration. CPU only.

The C3 / C5 goldens (mpc_cfg3_N100_H10, mpc_cfg5_N500_H20) come from the long-double oracle,
which runs the same Mehrotra iteration as the kernels. Two checks here do not use that code path:

1. Weak duality (oracle/certificate.py). From the golden's W, the dual point y_t = 1 / (R_t . w_t)
   and the LP-optimal z for that y (HiGHS dual simplex) give a lower bound g <= p*. The bound is
   re-evaluated in float64 from the dual formula. gap = f(W) - g >= 0 bounds the golden's
   suboptimality, whatever produced W.
2. A dense-KKT interior point (oracle/dense_ipm.py: the full (2HN+H)-square KKT matrix factored by
   LAPACK, no structure exploited) on four C3 windows. It is itself certified to 1e-9 (1 + |f*|).

Measured gaps of the goldens: <= 1e-9 on the small, cfg1 and cfg2 files; <= 1.1e-8 on cfg3 and
<= 7.6e-8 on cfg5. The oracle stops once its best iterate's scaled complementarity reaches
mu ~ 1e-10; its total complementarity is then ~1e-8 in objective units. These gaps are >= 20x
below the kernels' objective parity bar, 1e-6 + 1e-5 |f*| (tests/test_solver_gpu.py). The objective
is the parity quantity that transfers to the reference's SCS, which stops at eps 1e-4. W0 is
compared only where the optimum is unique; otherwise the optimal set is a face, and two interior
points stop at different points near its analytic centre.
"""
import glob
import os

import numpy as np
import pytest

from oracle import certificate as C
from oracle import dense_ipm

GOLD = os.path.join(os.path.dirname(__file__), "golden")

# per-file certified-gap bars (relative to 1 + |f*|), ~3x the measured worst case
GAP_BAR = {"mpc_cfg3_N100_H10.npz": 3e-8, "mpc_cfg5_N500_H20.npz": 2e-7}


@pytest.mark.parametrize("path", sorted(p for p in glob.glob(os.path.join(GOLD, "mpc_*_*.npz"))
                                        if "short" not in p and "kat" not in p))
def test_every_golden_is_certified_optimal(path):
    g = np.load(path)
    c, tau, _ = g["config"]
    bar = GAP_BAR.get(os.path.basename(path), 1e-9)
    for b in range(g["W"].shape[0]):
        r = C.certify(g["W"][b], g["w_prev"][b], g["yhat"][b], c, tau)
        # (the interior point stops at primal residuals <= 1e-8; the goldens' worst is 1.3e-10,
        # mpc_small_c0_t0.2 window 18 — 1e-12 before the initial multipliers went to 0.5)
        assert r["violation"] <= 1e-9, (b, r)
        assert -r["f"] == pytest.approx(g["obj"][b], abs=1e-12)      # the recorded problem.value
        assert r["gap"] >= -1e-11, (b, r)   # weak duality holds numerically (to the violation's
        #                                     order: window 18 above, -1.8e-12)
        assert r["gap"] <= bar * (1 + abs(r["f"])), (b, r)


def test_dense_kkt_ipm_pins_config3_goldens():
    g = np.load(os.path.join(GOLD, "mpc_cfg3_N100_H10.npz"))
    c, tau, _ = g["config"]
    for b in range(4):
        W, conv = dense_ipm.dense_ipm(g["w_prev"][b], g["yhat"][b], c, tau)
        assert conv
        r = C.certify(W, g["w_prev"][b], g["yhat"][b], c, tau)
        assert r["violation"] <= 1e-10 and 0 <= r["gap"] <= 1e-9 * (1 + abs(r["f"])), (b, r)
        # the golden objective sits within the golden's certified gap of the certified dense optimum
        assert abs(-r["f"] - g["obj"][b]) <= 2e-8, b
        # the parity-relevant statement: both are far inside the kernels' objective bar
        assert abs(-r["f"] - g["obj"][b]) <= 1e-2 * (1e-6 + 1e-5 * abs(g["obj"][b]))


def test_certificate_detects_a_suboptimal_point():
    """The bound is not vacuous: holding w_prev (feasible, not optimal) shows a large gap, and a
    point moved off the optimum by 1e-4 shows a gap of that order."""
    g = np.load(os.path.join(GOLD, "mpc_cfg3_N100_H10.npz"))
    c, tau, _ = g["config"]
    wp, y = g["w_prev"][0], g["yhat"][0]
    hold = np.tile(wp, (y.shape[0], 1))
    r = C.certify(hold, wp, y, c, tau)
    assert r["violation"] <= 1e-12 and r["gap"] > 1e-4
    W = g["W"][0].copy()
    i, j = np.argmax(W[-1]), np.argmin(W[-1])
    W[-1, i] -= 1e-4
    W[-1, j] += 1e-4                 # still feasible: budget kept, turnover of the last period < tau
    r2 = C.certify(W, wp, y, c, tau)
    assert r2["violation"] <= 1e-12 and r2["gap"] > 1e-7


def test_certificate_known_answers():
    """The reference's tests/test_mpc.py optima (mpc_kat.npz) certify to machine precision."""
    k = np.load(os.path.join(GOLD, "mpc_kat.npz"))
    r = C.certify(k["pref_W"], k["pref_wp"], k["pref_y"], 0.0, 0.2)
    assert abs(r["gap"]) <= 1e-12
    r = C.certify(k["cost_W"], k["cost_wp"], k["cost_y"], 10.0, 0.2)
    assert abs(r["gap"]) <= 1e-12
