"""GPU parity of the batched MPC solve kernel (through the C ABI) against the oracle goldens.

Parity bar: every problem optimal and feasible (sum w = 1 +- 1e-8, w >= -1e-9,
turnover <= tau + 1e-8); objective within 1e-6 + 1e-5 |f*| of the long-double oracle; applied
weights W[0] within 1e-3 of the oracle where the optimum is unique (cost > 0); for cost = 0 the
optimum is generally a face, so the objective criterion is the one that applies. (The reference's
own solver, SCS, stops at eps 1e-4.)
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import dense_ipm, solver as oracle
from koopman_mpc_portfolio_rebalancing_amd import MPCConfig, solve_mpc_log_utility, solve_mpc_log_utility_batched

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _solve(wp, y, c, tau, short=False, full=True, path=0, precision="auto"):
    H = y.shape[1]
    cfg = MPCConfig(horizon=H, cost_coeff=c, max_turnover=tau, allow_short=short, solver_path=path,
                    precision=precision)
    W, st, val = solve_mpc_log_utility_batched(torch.tensor(wp, device="cuda"), torch.tensor(y, device="cuda"),
                                               cfg, return_full=full)
    return W.cpu().numpy(), st.cpu().numpy(), val.cpu().numpy()


def _feasible(W, wp, tau, short, tol=1e-8):
    ok = np.allclose(W.sum(-1), 1.0, atol=tol)
    if not short:
        ok &= bool((W >= -1e-9).all())
    if tau > 0:
        prev = wp
        for t in range(W.shape[0]):
            ok &= np.abs(W[t] - prev).sum() <= tau + tol
            prev = W[t]
    return bool(ok)


# precision "auto" solves these golden batches (< KMPC_MIXED_MIN_B windows) in float64; "mixed"
# forces the float32 phase + float64 finish where the shape has it (the C3-shaped goldens)
@pytest.mark.parametrize("precision", ["auto", "mixed"])
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLD, "mpc_*_*.npz"))))
def test_solver_matches_golden(path, precision):
    if path.endswith("mpc_kat.npz"):
        pytest.skip("KATs tested separately")
    g = np.load(path)
    c, tau, short = g["config"]
    short = bool(short)
    W, st, val = _solve(g["w_prev"], g["yhat"], c, tau, short, precision=precision)
    # optimal everywhere, the shorting golden included (pinned: every window reaches "optimal" since
    # the shorting refinement threshold REFINE_MU_SHORT; a status regression fails here)
    assert (st == 0).all(), st
    for b in range(W.shape[0]):
        assert _feasible(W[b], g["w_prev"][b], tau, short), b
    f_ref = g["obj"]
    assert np.abs(val - f_ref).max() <= 1e-6 + 1e-5 * np.abs(f_ref).max()
    # the reported value is problem.value at the returned W
    for b in range(min(W.shape[0], 4)):
        assert val[b] == pytest.approx(dense_ipm.reference_objective(W[b], g["w_prev"][b], g["yhat"][b], c), abs=1e-12)
    if c > 0 and not short:
        assert np.abs(W[:, 0] - g["W"][:, 0]).max() < 1e-3


@pytest.mark.parametrize("name,precision", [("mpc_cfg3_N100_H10.npz", "auto"), ("mpc_cfg3_N100_H10.npz", "mixed"),
                                            ("mpc_cfg5_N500_H20.npz", "auto"), ("mpc_cfg1_N10_H5.npz", "auto")])
def test_device_solutions_are_certified_optimal(name, precision):
    """The device's own W, certified by weak duality (oracle/certificate.py: the LP-optimal dual z
    for y = 1 / (R.w), no interior-point code): gap <= the objective parity bar 1e-6 + 1e-5 |f*|.
    This is W-parity as distance to the optimal set: it holds wherever on the optimal face the
    interior point stops, so it transfers to any solver that reaches the optimum (SCS included)."""
    from oracle import certificate
    g = np.load(os.path.join(GOLD, name))
    c, tau, _ = g["config"]
    W, st, val = _solve(g["w_prev"], g["yhat"], c, tau, precision=precision)
    assert (st == 0).all()
    for b in range(W.shape[0]):
        r = certificate.certify(W[b], g["w_prev"][b], g["yhat"][b], c, tau)
        assert r["violation"] <= 1e-8 and -1e-12 <= r["gap"] <= 1e-6 + 1e-5 * abs(r["f"]), (b, r)
        assert -r["f"] == pytest.approx(val[b], abs=1e-12)


def test_reference_test_mpc_cases_on_device():
    """tests/test_mpc.py of the reference, through the per-window drop-in (mpc.py:27 signature)."""
    W, info = solve_mpc_log_utility(np.ones(5) / 5, np.zeros((3, 5)), MPCConfig(horizon=3, cost_coeff=0.0))
    assert info["status"] == "optimal" and W.shape == (3, 5)
    for t in range(3):
        assert np.isclose(W[t].sum(), 1.0) and (W[t] >= -1e-5).all()
    W, _ = solve_mpc_log_utility(np.array([0.5, 0.5]), np.array([[0.1, 0.0]]), MPCConfig(horizon=1, cost_coeff=0.0))
    assert W[0, 0] > 0.5 and W[0, 1] < 0.5
    assert np.abs(W[0] - [0.6, 0.4]).max() < 1e-6
    W, _ = solve_mpc_log_utility(np.array([1.0, 0.0]), np.array([[0.0, 0.01]]), MPCConfig(horizon=1, cost_coeff=10.0))
    assert np.allclose(W[0], [1.0, 0.0], atol=1e-6)


def test_fallback_statuses_on_device():
    y = np.array([[[0.01, 0.0]], [[np.nan, 0.0]]], np.float32)
    wp = np.array([[1.0, 1.0], [0.5, 0.5]])
    W, st, val = _solve(wp, y, 1e-3, 0.2)
    assert st[0] == 2 and st[1] == 4                    # infeasible, solver_error
    assert np.array_equal(W[:, 0], wp) and np.isnan(val).all()
    W, st, val = _solve(np.array([[0.5, 0.5]]), y[:1], 0.0, 0.0, short=True)
    assert st[0] == 3 and np.array_equal(W[0, 0], [0.5, 0.5])
    _, info = solve_mpc_log_utility(np.array([1.0, 1.0]), np.array([[0.01, 0.0]]), MPCConfig(horizon=1))
    assert info == {"status": "infeasible", "value": None}


@pytest.mark.parametrize("N,H", [(1, 3), (63, 4), (64, 5), (65, 6), (129, 2), (300, 7), (20, 12),
                                 (100, 10), (64, 10),                  # exact-H, constant-case kernel
                                 (65, 10), (103, 10), (104, 10),       # QL variant (N < 104) and its edges
                                 (100, 9), (103, 7),                   # generic QL variant (ragged H)
                                 (200, 10), (256, 5),                  # constant-case, 256 threads
                                 (215, 10), (216, 10),                 # 256-thread QL variant edges
                                 (100, 21), (200, 21), (30, 15),       # HM = 21: exact and ragged H
                                 (500, 20), (700, 3), (520, 10), (1000, 10)])   # 512- and 1024-thread variants
def test_ragged_shapes_match_oracle(N, H):
    rng = np.random.default_rng(N * 31 + H)
    B = 6
    wp = rng.dirichlet(np.ones(N), B)
    y = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
    W, st, val = _solve(wp, y, 1e-3, 0.3)
    # run-to-run bit-identical (a barrier race in the turnover-cap update showed up here first)
    W2, st2, val2 = _solve(wp, y, 1e-3, 0.3)
    assert np.array_equal(W, W2) and np.array_equal(st, st2) and np.array_equal(val, val2, equal_nan=True)
    Wo, sto, valo, _ = oracle.solve_batch(wp, y, 1e-3, 0.3)
    assert (st <= 1).all() and (sto <= 1).all()
    assert np.abs(val - valo).max() <= 1e-6 + 1e-5 * np.abs(valo).max()
    assert np.abs(W[:, 0] - Wo[:, 0]).max() < 1e-3


@pytest.mark.parametrize("N,H,case", [(10, 5, 0), (16, 5, 1), (1, 3, 0), (13, 4, 2), (3, 2, 3),   # 16-lane groups
                                      (17, 5, 0), (30, 5, 1), (32, 10, 0), (20, 7, 2), (25, 10, 3),  # 32-lane groups
                                      (31, 1, 0), (10, 5, 4)])
def test_packed_small_windows_match_oracle(N, H, case):
    """N <= 32: 4 (16-lane groups: N <= 16, H <= 5) or 2 (32-lane groups) windows per wave. A batch
    that does not fill the last wave, a non-finite and an infeasible window between solved ones
    (their groups leave the iteration early while their neighbours keep iterating), against the
    long-double oracle and the one-window-per-wave kernels (KMPC_PATH_REGISTER_UNPACKED)."""
    from koopman_mpc_portfolio_rebalancing_amd import _lib
    c, tau, short = [(1e-3, 0.2, False), (0.0, 0.0, False), (1e-3, 0.0, False), (0.0, 0.3, False),
                     (5e-3, 0.0, True)][case]
    rng = np.random.default_rng(100 * N + H + case)
    B = 11
    wp = rng.dirichlet(np.ones(N), B)
    if short:
        wp = wp * 1.5 - 0.5 / N
    y = rng.normal(5e-4, 0.02, (B, H, N)).astype(np.float32)
    y[4, H - 1, 0] = np.nan                     # solver_error inside a pack
    if tau > 0 and N > 1:
        wp[6] = 0.0
        wp[6, 0] = 3.0                          # sum(w_prev) = 3: the cap makes the budget unreachable
    path = _lib.PATH_REGISTER   # (packed at any batch size — AUTO packs from KMPC_PACK_MIN_B — and no presolve)
    W, st, val = _solve(wp, y, c, tau, short, path=path)
    W2, st2, val2 = _solve(wp, y, c, tau, short, path=path)
    assert np.array_equal(W, W2) and np.array_equal(st, st2) and np.array_equal(val, val2, equal_nan=True)
    Wu, stu, valu = _solve(wp, y, c, tau, short, path=_lib.PATH_REGISTER_UNPACKED)
    Wo, sto, valo, _ = oracle.solve_batch(wp, y, c, tau, allow_short=short)
    assert np.array_equal(st <= 1, sto <= 1) and np.array_equal(st <= 1, stu <= 1), (st, sto, stu)
    assert st[4] == 4 and np.array_equal(W[4], np.tile(wp[4], (H, 1))) and np.isnan(val[4])
    if tau > 0 and N > 1:
        assert st[6] == 2 and np.array_equal(W[6], np.tile(wp[6], (H, 1)))
    ok = sto <= 1
    assert ok.sum() >= 8
    bar = 1e-6 + 1e-5 * np.abs(valo[ok]).max()
    assert np.abs(val[ok] - valo[ok]).max() <= bar and np.abs(val[ok] - valu[ok]).max() <= bar
    for b in np.flatnonzero(ok):
        assert _feasible(W[b], wp[b], tau, short), b
    if c > 0 and not short:
        assert np.abs(W[ok, 0] - Wo[ok, 0]).max() < 1e-3


def test_full_size_properties_and_determinism():
    """cfg3 shape at 8192 windows: every window optimal and feasible, never worse than holding
    (W = tile(w_prev) is feasible), bit-identical on a second launch."""
    rng = np.random.default_rng(7)
    B, N, H = 8192, 100, 10
    wp = rng.dirichlet(np.ones(N), B)
    y = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
    W, st, val = _solve(wp, y, 1e-3, 0.2)
    W2, st2, val2 = _solve(wp, y, 1e-3, 0.2)
    assert np.array_equal(W, W2) and np.array_equal(val, val2)
    assert (st == 0).all()
    assert np.abs(W.sum(-1) - 1).max() < 1e-8 and W.min() > -1e-9
    turn = np.abs(np.diff(np.concatenate([wp[:, None], W], 1), axis=1)).sum(-1)
    assert turn.max() <= 0.2 + 1e-8
    hold = np.log(np.exp(y).astype(np.float64) @ wp[:, :, None])[..., 0].sum(-1)   # R in float32 (mpc.py:55)
    assert (val >= hold - 1e-9).all()


def test_simplex_presolve_matches_ipm_and_oracle():
    """c = tau = 0, no short (BASELINE configs[1]): the closed-form presolve returns the IPM's
    optimum — the argmax vertex per period, the centre of the face on exact ties."""
    from koopman_mpc_portfolio_rebalancing_amd import _lib
    rng = np.random.default_rng(5)
    B, N, H = 64, 30, 5
    wp = rng.dirichlet(np.ones(N), B)
    y = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
    y[0, 1, [3, 7]] = y[0, 1].max() + 0.01          # an exact two-way tie
    y[1, :, :] = 0.0                                 # flat window: every asset tied
    W, st, val = _solve(wp, y, 0.0, 0.0)
    assert (st == 0).all()
    am = y.argmax(-1)
    for b in range(2, B):
        assert np.array_equal(W[b], np.eye(N)[am[b]])
    assert np.array_equal(W[0, 1, [3, 7]], [0.5, 0.5]) and W[0, 1].sum() == 1.0
    assert np.allclose(W[1], 1.0 / N, rtol=0, atol=1e-15)
    for b in range(4):
        assert val[b] == pytest.approx(dense_ipm.reference_objective(W[b], wp[b], y[b], 0.0), abs=1e-12)
    # the interior-point kernels (per-call path KMPC_PATH_REGISTER: no presolve) reach the same optimum
    Wi, sti, vali = _solve(wp, y, 0.0, 0.0, path=_lib.PATH_REGISTER)
    assert (sti == 0).all()
    # exact vs interior point stopped at mu 1e-9 (scaled): never worse, within the parity bar
    assert (val >= vali - 1e-12).all() and np.abs(val - vali).max() < 1e-7
    assert np.abs(W[2:] - Wi[2:]).max() < 1e-3        # (near-ties keep the IPM iterate ~1e-5 inside)
    Wo, sto, valo, _ = oracle.solve_batch(wp, y, 0.0, 0.0)
    assert (val >= valo - 1e-12).all() and np.abs(val - valo).max() < 1e-8
    # non-finite input: solver_error with the reference fallback
    y2 = y[:2].copy(); y2[1, 0, 0] = np.nan
    W2, st2, val2 = _solve(wp[:2], y2, 0.0, 0.0)
    assert st2.tolist() == [0, 4] and np.isnan(val2[1]) and np.array_equal(W2[1], np.tile(wp[1], (H, 1)))


def test_randomized_sweep_of_solver_paths():
    """Random (N, H, cost, cap, short) draws across every dispatch path — register kernels (64 /
    128 / 256 threads, constant-case and generic, exact and ragged H), the large-window kernel and
    the simplex presolve — against the long-double oracle (objective bar of the module docstring;
    W[0] where the optimum is unique)."""
    rng = np.random.default_rng(2024)
    shapes = [(10, 5), (30, 5), (64, 10), (100, 10), (100, 7), (150, 10), (256, 10), (40, 2),
              (300, 5), (80, 12), (120, 20), (20, 1)]
    cases = [(1e-3, 0.2, False), (0.0, 0.0, False), (1e-3, 0.0, False), (0.0, 0.3, False),
             (5e-3, 0.5, True), (1e-3, 0.0, True)]
    for k, (N, H) in enumerate(shapes):
        c, tau, short = cases[k % len(cases)]
        B = 3
        wp = rng.dirichlet(np.ones(N), B)
        if short:
            wp = wp * 1.5 - 0.5 / N
        y = rng.normal(5e-4, 0.02, (B, H, N)).astype(np.float32)
        W, st, val = _solve(wp, y, c, tau, short)
        Wo, sto, valo, _ = oracle.solve_batch(wp, y, c, tau, allow_short=short)
        assert np.array_equal(st <= 1, sto <= 1), (N, H, c, tau, short, st, sto)
        ok = sto <= 1
        assert np.abs(val[ok] - valo[ok]).max() <= 1e-6 + 1e-5 * np.abs(valo[ok]).max(), (N, H, c, tau, short)
        for b in np.flatnonzero(ok):
            assert _feasible(W[b], wp[b], tau, short), (N, H, c, tau, short, b)
        if c > 0 and not short:
            assert np.abs(W[ok, 0] - Wo[ok, 0]).max() < 1e-3, (N, H, c, tau)


def test_gross_returns_bit_exact():
    """kmpc_gross_returns (the kernels' R = np.exp(yhat), kmpc_npexp.h) against numpy's float32 exp
    on every 5th float32 bit pattern (859M inputs: all exponents, saturation, NaN / inf) and a
    dense sweep of log-return-sized inputs."""
    import ctypes
    from koopman_mpc_portfolio_rebalancing_amd import _lib
    L = _lib.load()
    chunk = 1 << 26
    for start in range(0, 1 << 32, chunk * 5):
        n = min(chunk, ((1 << 32) - start + 4) // 5)
        bits = torch.arange(start, start + 5 * n, 5, dtype=torch.int64, device="cuda").to(torch.int32)
        x = bits.view(torch.float32)
        R = torch.empty_like(x)
        _lib.check(L.kmpc_gross_returns(n, x.data_ptr(), R.data_ptr(), None))
        xh, Rh = x.cpu().numpy(), R.cpu().numpy()
        with np.errstate(over="ignore", invalid="ignore"):
            ref = np.exp(xh)
        same = (Rh.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(Rh) & np.isnan(ref))
        assert same.all(), (start, xh[~same][:4], Rh[~same][:4], ref[~same][:4])
    x = torch.linspace(-0.3, 0.3, 1 << 24, device="cuda")
    R = torch.empty_like(x)
    _lib.check(L.kmpc_gross_returns(x.numel(), x.data_ptr(), R.data_ptr(), None))
    assert np.array_equal(R.cpu().numpy().view(np.uint32), np.exp(x.cpu().numpy()).view(np.uint32))


def test_float32_gross_return_ties():
    """The program the reference solves sees R = np.exp(yhat) in float32 (mpc.py:55): distinct yhat
    that round to one R are tied assets. Presolve (c = tau = 0): the face of the tied maximum, not
    the argmax of yhat. Interior point with a cap: flat objective, centre w_prev (a float64
    exp(yhat) would move to the cap, [0.6, 0.4]). Both against the oracle fed numpy's R."""
    a = np.float32(0.01)
    b = np.nextafter(a, np.float32(0))
    c_ = np.nextafter(b, np.float32(0))
    assert np.exp(np.array([a, b, c_]))[0] == np.exp(np.array([a, b, c_]))[2]
    y = np.array([[[a, b, c_, 0.0]], [[0.0, b, 0.0, a]]], np.float32)          # [B=2, H=1, N=4]
    wp = np.full((2, 4), 0.25)
    W, st, val = _solve(wp, y, 0.0, 0.0)                                     # presolve
    assert (st == 0).all()
    assert np.array_equal(W[0, 0], [1 / 3, 1 / 3, 1 / 3, 0.0]) and np.array_equal(W[1, 0], [0.0, 0.5, 0.0, 0.5])
    R = np.exp(y).astype(np.float64)
    assert val[0] == pytest.approx(np.log(R[0, 0, 0]), abs=1e-15) and val[1] == np.log(R[1, 0, 1])
    Wo, sto, valo, _ = oracle.solve_batch(wp, y, 0.0, 0.0)
    assert np.abs(val - valo).max() < 1e-12
    y2 = np.array([[[a, b]]], np.float32)
    W2, st2, val2 = _solve(np.array([[0.5, 0.5]]), y2, 0.0, 0.2)             # interior point, cap 0.2
    Wo2, sto2, valo2, _ = oracle.solve_batch(np.array([[0.5, 0.5]]), y2, 0.0, 0.2)
    assert st2[0] == 0 and sto2[0] == 0
    assert np.abs(W2[0, 0] - 0.5).max() < 1e-6 and np.abs(Wo2[0, 0] - 0.5).max() < 1e-6
    assert val2[0] == pytest.approx(np.log(np.float64(np.exp(a))), abs=1e-15)


@pytest.mark.parametrize("N,H,c,tau,path", [(3, 2, 0.0, 0.0, 0),      # presolve, register fast path
                                            (80, 20, 0.0, 0.0, 0),    # presolve, general loop
                                            (3, 2, 1e-3, 0.2, 0),     # packed interior point
                                            (100, 10, 1e-3, 0.2, 0),  # register kernel (C3 case)
                                            (70, 7, 0.0, 0.0, 1),     # register kernel, no presolve
                                            (300, 12, 1e-3, 0.2, 0)])  # large-window kernel
def test_underflowed_period_is_infeasible(N, H, c, tau, path):
    """R = np.exp(yhat) is 0 in float32 for yhat <= -103.97 (mpc.py:55). A period where every R is
    0 has R.w = 0 on the whole simplex, and the reference's exp cone exp(u) <= R.w has no
    solution: cvxpy reports infeasible, the strategy holds w_prev (mpc.py:113-115). Every path
    reports it the same way as the oracle, next to an ordinary window."""
    rng = np.random.default_rng(N + H)
    wp = rng.dirichlet(np.ones(N), 2)
    y = rng.normal(5e-4, 0.015, (2, H, N)).astype(np.float32)
    y[1, H - 1, :] = -110.0
    y[1, 0, 0] = -200.0
    W, st, val = _solve(wp, y, c, tau, path=path)
    Wo, sto, valo, _ = oracle.solve_batch(wp, y, c, tau)
    assert st[1] == 2 and sto[1] == 2, (st, sto)
    assert np.array_equal(W[1], np.tile(wp[1], (H, 1))) and np.isnan(val[1])
    assert st[0] == 0 and abs(val[0] - valo[0]) <= 1e-6 + 1e-5 * abs(valo[0])


@pytest.mark.parametrize("N,H,B", [(30, 15, 1600), (300, 12, 1100)])
def test_large_window_slot_reuse(N, H, B):
    """The large-window kernel runs a persistent grid (768 / 512 workgroups) whose workgroups solve
    window after window in the same workspace slab and LDS: with B past the slot count, windows
    solved later by a reused workgroup must equal the same windows solved alone, bit for bit, and
    a sample must match the oracle."""
    rng = np.random.default_rng(N + H + B)
    wp = rng.dirichlet(np.ones(N), B)
    y = rng.normal(5e-4, 0.015, (B, H, N)).astype(np.float32)
    W, st, val = _solve(wp, y, 1e-3, 0.3, full=False)
    assert (st <= 1).all()
    for b in (0, 767, 768, 1099, B - 1):
        if b >= B:
            continue
        W1, st1, val1 = _solve(wp[b:b + 1], y[b:b + 1], 1e-3, 0.3, full=False)
        assert st1[0] == st[b] and np.array_equal(W1[0], W[b]) and val1[0] == val[b], b
    idx = np.array([1, 800, B - 2])
    Wo, sto, valo, _ = oracle.solve_batch(wp[idx], y[idx], 1e-3, 0.3)
    assert (sto <= 1).all()
    assert np.abs(val[idx] - valo).max() <= 1e-6 + 1e-5 * np.abs(valo).max()
    assert np.abs(W[idx] - Wo[:, 0]).max() < 1e-3


@pytest.mark.parametrize("N,H,c,tau,path", [(3, 2, 0.0, 0.0, 0),      # presolve, register fast path
                                            (80, 20, 0.0, 0.0, 0),    # presolve, general loop
                                            (3, 2, 1e-3, 0.2, 0),     # packed interior point
                                            (100, 10, 1e-3, 0.2, 0),  # C3 case (float32 phase + float64)
                                            (100, 10, 1e-3, 0.2, -1),  # C3 case, float64 only
                                            (70, 7, 0.0, 0.0, 1),     # register kernel, no presolve
                                            (300, 12, 1e-3, 0.2, 0)])  # large-window kernel
def test_tiny_gross_return_period_is_solved(N, H, c, tau, path):
    """a period whose every yhat is ~ -50 has R ~ 2e-22 > 0. The reference's program
    is feasible and optimal there (log(R.w) is finite), but m = R - 1 rounds to -1 in float64, so
    the interior points used to report it infeasible while the presolve said optimal. Every path now
    solves such a period on R / sum(R) (TINY_PERIOD) and adds log sum(R) back: the same status on
    every path (optimal), the oracle's objective, and the shift property — the window equals the
    unshifted one with that period's objective lowered by 50 (float32 rounding of yhat - 50 aside)."""
    rng = np.random.default_rng(N * 7 + H)
    wp = rng.dirichlet(np.ones(N), 2)
    y = rng.normal(5e-4, 0.015, (2, H, N)).astype(np.float32)
    y2 = y.copy()
    y2[1, H - 1, :] -= 50.0
    prec = "f64" if path < 0 else "auto"
    path = max(path, 0)
    W, st, val = _solve(wp, y2, c, tau, path=path, precision=prec)
    Wu, stu, valu = _solve(wp, y, c, tau, path=path, precision=prec)
    Wo, sto, valo, _ = oracle.solve_batch(wp, y2, c, tau)
    assert (st == 0).all() and (sto == 0).all(), (st, sto)
    assert np.abs(val - valo).max() <= 1e-6 + 1e-5 * np.abs(valo).max()
    assert abs((val[1] + 50.0) - valu[1]) < 5e-5            # float32 yhat - 50 keeps ~4e-6 of yhat
    assert np.array_equal(W[0], Wu[0])                       # the other window is untouched
    if c > 0:
        assert np.abs(W[1, 0] - Wu[1, 0]).max() < 1e-3


@pytest.mark.parametrize("name", ["mpc_cfg1_N10_H5.npz", "mpc_cfg3_N100_H10.npz", "mpc_cfg5_N500_H20.npz",
                                  "mpc_small_c1e-3_t0.2.npz", "mpc_small_c1e-3_t0.npz"])
def test_iteration_counts_follow_the_oracle(name):
    """The kernels run the oracle's iteration — initial point (multipliers 0.5), step rule (0.995 of
    the boundary without shorting), centring rule (sigma <= 0.2 with the cap), stopping rule
    (kmpc_solve_kernel.h, oracle/kmpc_oracle.c) — so the float64 solve's iteration counts track the
    long-double oracle's at the same stopping tolerance, 1e-9 (the goldens were made at the oracle's
    default 1e-11, about one iteration more; the kernels refine to 1e-5 instead of 1e-7 and round
    in float64: a window may differ by an iteration or two, the mean by well under one)."""
    from oracle import solver as oracle
    g = np.load(os.path.join(GOLD, name))
    c, tau, short = g["config"]
    _, sto, _, ref = oracle.solve_batch(g["w_prev"], g["yhat"], c, tau, bool(short), tol=1e-9, precision="ld")
    assert (sto == 0).all()
    H = g["yhat"].shape[1]
    cfg = MPCConfig(horizon=H, cost_coeff=c, max_turnover=tau, allow_short=bool(short), precision="f64")
    W, st, val, it = solve_mpc_log_utility_batched(torch.tensor(g["w_prev"], device="cuda"),
                                                   torch.tensor(g["yhat"], device="cuda"), cfg, with_iters=True)
    it = it.cpu().numpy().astype(np.int64)
    ref = ref.astype(np.int64)
    assert (st.cpu().numpy() == 0).all()
    print(name, "device", it.mean(), "oracle", ref.mean(), "max |d|", np.abs(it - ref).max())
    # (measured: mean differences 0-0.19, per window at most 1)
    assert abs(it.mean() - ref.mean()) <= 0.5
    assert np.abs(it - ref).max() <= 2
