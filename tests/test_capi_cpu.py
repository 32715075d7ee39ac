"""The C ABI boundary without a GPU: libkmpc.so loads, exports every function include/kmpc.h
declares, and the ctypes mirrors match the C struct layouts (checked by compiling the header)."""
import ctypes
import inspect
import os
import re
import subprocess

import numpy as np
import pytest

from koopman_mpc_portfolio_rebalancing_amd import _lib
import koopman_mpc_portfolio_rebalancing_amd as pkg

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "kmpc.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kmpc_[a-z_]+)\s*\(", src)))


def test_library_exports_every_header_function():
    lib = _lib.load()
    names = header_functions()
    assert set(names) == set(_lib.EXPORTED_SYMBOLS)
    for n in names:
        assert hasattr(lib, n), n
    assert lib.kmpc_version().decode().startswith(f"kmpc {_lib.ABI_VERSION} ")
    assert lib.kmpc_strerror(_lib.KMPC_OK).decode() == "ok"
    assert lib.kmpc_strerror(100 + 1).decode() == "optimal_inaccurate"


def test_argument_errors_need_no_gpu():
    lib = _lib.load()
    d = _lib.SolveDesc()
    d.B, d.N, d.H = 1, 5, 0
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -1
    d.H, d.N = 40, 5
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -2
    d.H, d.B = 5, 0
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == 0
    d.cost_coeff = -1e-3                   # not convex: cvxpy raises, the boundary rejects it
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -1
    d.cost_coeff, d.path = 0.0, 7           # unknown solver path
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -1
    d.path, d.precision = 0, 3              # unknown precision
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -1
    d.precision, d.mu_handoff = 0, 1.5       # a handoff past mu = 1 is no handoff
    assert lib.kmpc_solve(ctypes.byref(d), None, None, None, None, None, None, None, 0, None) == -1
    d.mu_handoff = 0.0
    # the mixed-precision pair (C3 shape) needs a 64 B record header per window (the iterate goes
    # from the float32 phase to the float64 finish on chip), the whole batch at once
    d.B, d.N, d.H, d.cost_coeff, d.max_turnover, d.precision = 1000, 100, 10, 1e-3, 0.2, 2   # MIXED
    rec = 64
    assert lib.kmpc_workspace_bytes(None, ctypes.byref(d)) == 1000 * rec
    d.B = 1 << 20
    assert lib.kmpc_workspace_bytes(None, ctypes.byref(d)) == (1 << 20) * rec
    d.B = 1000
    d.precision = 1
    assert lib.kmpc_workspace_bytes(None, ctypes.byref(d)) == 0
    d.precision = 0                          # AUTO: float64 below KMPC_MIXED_MIN_B windows, the pair from it
    assert lib.kmpc_workspace_bytes(None, ctypes.byref(d)) == 0
    d.B = _lib.MIXED_MIN_B
    assert lib.kmpc_workspace_bytes(None, ctypes.byref(d)) == _lib.MIXED_MIN_B * rec
    d.B, d.N, d.H, d.cost_coeff, d.max_turnover, d.precision = 0, 5, 5, 0.0, 0.0, 0
    assert lib.kmpc_gross_returns(0, None, None, None) == 0
    assert lib.kmpc_gross_returns(4, None, None, None) == -1
    bt = _lib.BacktestDesc(2, 3, 4, 1e-3)
    assert lib.kmpc_backtest_step(ctypes.byref(bt), 4, None, None, None, None, None, None) == -1   # step >= S
    assert lib.kmpc_backtest_step(ctypes.byref(bt), 0, None, None, None, None, None, None) == -1   # null arrays
    assert lib.kmpc_backtest_metrics(None, None, None, None) == -1
    # kmpc_backtest_run: argument checks, then the shape check (n_steps = 0: no launch)
    sd = _lib.SolveDesc()
    sd.B, sd.N, sd.H, sd.cost_coeff, sd.max_turnover = 0, 100, 10, 1e-3, 0.2
    btr = _lib.BacktestDesc(64, 100, 20, 1e-3)
    run = lambda *a: lib.kmpc_backtest_run(ctypes.byref(btr), ctypes.byref(sd), *a, *([None] * 6), None)
    assert run(0, 0, None, None, 0) == 0                      # the C3 shape in float64: supported
    assert run(15, 6, None, None, 0) == -1                    # past the history's S rows
    assert run(0, 2, None, None, 0) == -1                     # null arrays
    assert run(0, 0, None, None, 1) == -1                     # more realized rows than steps
    sd.precision = 2                                          # MIXED: the per-step batch runs the pair
    assert run(0, 0, None, None, 0) == -2
    sd.precision, sd.H = 0, 5                                 # H = 5 constant-case kernels: supported
    assert run(0, 0, None, None, 0) == 0
    sd.H = 7                                                  # another horizon: no persistent kernel
    assert run(0, 0, None, None, 0) == -2
    sd.H, sd.N, btr.N = 5, 20, 20                             # N <= 32: the packed kernels' persistent form
    assert run(0, 0, None, None, 0) == 0
    sd.H = 3                                                  # a ragged packed horizon: no persistent form
    assert run(0, 0, None, None, 0) == -2
    sd.N, btr.N = 100, 100
    sd.H, sd.cost_coeff = 10, -1.0                            # the solve's own checks apply
    assert run(0, 0, None, None, 0) == -1
    bt.P = 0
    assert lib.kmpc_backtest_metrics(ctypes.byref(bt), None, None, None) == 0
    mv = _lib.MvDesc()
    mv.B, mv.N, mv.H = 1, 20, 0
    assert lib.kmpc_solve_mv(ctypes.byref(mv), None, None, 0, None, None, None, None, None, None) == -1
    mv.H, mv.N = 1, 1025                                      # H * N > KMPC_MV_MAX_HN
    assert lib.kmpc_solve_mv(ctypes.byref(mv), None, None, 0, None, None, None, None, None, None) == -2
    mv.N, mv.B = 20, 0
    assert lib.kmpc_solve_mv(ctypes.byref(mv), None, None, 0, None, None, None, None, None, None) == 0
    assert lib.kmpc_rolling_moments(1, 10, 3, 0, None, 3, None, None, None, None, None, None, None) == -1
    assert lib.kmpc_rolling_moments(0, 10, 3, 60, None, 3, None, None, None, None, None, None, None) == 0


def test_struct_layouts_match_header(tmp_path):
    prog = tmp_path / "layout.c"
    prog.write_text(f'''#include <stdio.h>
#include <stddef.h>
#include "{HEADER}"
int main(void) {{
  printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(kmpc_solve_desc), offsetof(kmpc_solve_desc, tol),
         offsetof(kmpc_solve_desc, return_full_W), offsetof(kmpc_solve_desc, max_turnover),
         offsetof(kmpc_solve_desc, path), offsetof(kmpc_solve_desc, precision),
         offsetof(kmpc_solve_desc, mu_handoff));
  printf("%zu %zu %zu\\n", sizeof(kmpc_mlp), offsetof(kmpc_mlp, weight), offsetof(kmpc_mlp, bias));
  printf("%zu %zu %zu %zu %zu\\n", sizeof(kmpc_rollout_desc), offsetof(kmpc_rollout_desc, encoder),
         offsetof(kmpc_rollout_desc, lista_thresh), offsetof(kmpc_rollout_desc, decoder),
         offsetof(kmpc_rollout_desc, std));
  printf("%zu %zu %zu\\n", offsetof(kmpc_rollout_desc, obs_ld), offsetof(kmpc_rollout_desc, dtype),
         offsetof(kmpc_rollout_desc, latent_unfused));
  printf("%zu %zu\\n", sizeof(kmpc_backtest_desc), offsetof(kmpc_backtest_desc, cost_coeff));
  printf("%zu %zu %zu %zu\\n", sizeof(kmpc_mv_desc), offsetof(kmpc_mv_desc, gamma),
         offsetof(kmpc_mv_desc, tol), offsetof(kmpc_mv_desc, return_full_W));
  return 0;
}}
''')
    exe = tmp_path / "layout"
    subprocess.run(["gcc", str(prog), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    S, M, R, Bt, Mv = _lib.SolveDesc, _lib.Mlp, _lib.RolloutDesc, _lib.BacktestDesc, _lib.MvDesc
    expect = [ctypes.sizeof(S), S.tol.offset, S.return_full_W.offset, S.max_turnover.offset, S.path.offset,
              S.precision.offset, S.mu_handoff.offset,
              ctypes.sizeof(M), M.weight.offset, M.bias.offset,
              ctypes.sizeof(R), R.encoder.offset, R.lista_thresh.offset, R.decoder.offset, R.std.offset,
              R.obs_ld.offset, R.dtype.offset, R.latent_unfused.offset,
              ctypes.sizeof(Bt), Bt.cost_coeff.offset,
              ctypes.sizeof(Mv), Mv.gamma.offset, Mv.tol.offset, Mv.return_full_W.offset]
    assert [int(x) for x in out] == expect


def test_reference_api_surface():
    """Field names/defaults of the reference dataclasses (mpc.py:17-25, backtest.py:22-30) and the
    public signatures the reference's callers use."""
    c = pkg.MPCConfig()
    assert (c.horizon, c.gamma, c.cost_coeff, c.max_turnover, c.allow_short, c.solver) == \
        (5, 0.0, 0.001, 0.2, False, "ECOS")
    b = pkg.BacktestConfig()
    assert (b.initial_capital, b.horizon, b.rebalance_freq, b.cost_coeff, b.risk_free_rate, b.allow_short) == \
        (10000.0, 5, 1, 0.001, 0.0, False)
    assert list(inspect.signature(pkg.solve_mpc_log_utility).parameters) == \
        ["current_weights", "predicted_log_returns", "config"]
    assert list(inspect.signature(pkg.run_backtest).parameters) == ["strategy", "env", "config", "verbose"]
    assert list(inspect.signature(pkg.KoopmanMPCStrategy.__init__).parameters) == \
        ["self", "model", "mpc_config", "device"]
    assert list(inspect.signature(pkg.KoopmanMPCStrategy.rebalance).parameters) == \
        ["self", "t", "current_weights", "env", "lookback_window"]
    assert list(inspect.signature(pkg.solve_mpc_mean_variance).parameters) == \
        ["current_weights", "predicted_log_returns", "cov_matrix", "config"]
    from koopman_mpc_portfolio_rebalancing_amd.baselines import MarkowitzStrategy
    m = MarkowitzStrategy(risk_aversion=2.0, cost_coeff=0.01)     # reference tests/test_baselines.py:22-27
    assert (m.risk_aversion, m.cost_coeff, m.mpc_config.gamma, m.mpc_config.horizon) == (2.0, 0.01, 2.0, 1)
    assert list(inspect.signature(MarkowitzStrategy.__init__).parameters) == \
        ["self", "risk_aversion", "cost_coeff", "allow_short"]


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.KmpcError):
        pkg.solve_mpc_log_utility(np.array([0.5, 0.5]), np.zeros((1, 2), np.float32), pkg.MPCConfig(horizon=1))
    with pytest.raises(_lib.KmpcError):
        pkg.solve_mpc_log_utility_batched(torch.ones(1, 2, dtype=torch.float64) / 2, torch.zeros(1, 1, 2),
                                          pkg.MPCConfig(horizon=1))
    with pytest.raises(_lib.KmpcError):
        pkg.solve_mpc_mean_variance(np.array([0.5, 0.5]), np.zeros((1, 2)), np.eye(2), pkg.MPCConfig(horizon=1))
    from koopman_mpc_portfolio_rebalancing_amd.baselines import MarkowitzStrategy
    with pytest.raises(_lib.KmpcError):
        MarkowitzStrategy().rebalance(10, np.array([0.5, 0.5]), None)


def test_compat_shims_expose_reference_module_names():
    """`from mpc import ...` / `from backtest import ...` resolve to the engine via compat/ (INTEGRATION.md)."""
    import importlib
    import sys
    from koopman_mpc_portfolio_rebalancing_amd import compat
    saved = {k: sys.modules.pop(k) for k in ("mpc", "backtest") if k in sys.modules}
    sys.path.insert(0, compat.PATH)
    try:
        mpc = importlib.import_module("mpc")
        backtest = importlib.import_module("backtest")
        import koopman_mpc_portfolio_rebalancing_amd as k
        assert mpc.solve_mpc_log_utility is k.solve_mpc_log_utility and mpc.MPCConfig is k.MPCConfig
        for name in ("BacktestConfig", "Strategy", "BuyAndHoldStrategy", "KoopmanMPCStrategy",
                     "run_backtest", "calculate_metrics", "solve_mpc_log_utility", "MPCConfig"):
            assert getattr(backtest, name) is getattr(k, name)
        assert mpc.MPCConfig().solver == "ECOS" and mpc.MPCConfig().horizon == 5
    finally:
        sys.path.remove(compat.PATH)
        for name in ("mpc", "backtest"):
            sys.modules.pop(name, None)
        sys.modules.update(saved)


def test_python_constants_match_the_header():
    """The ctypes layer's enum values (_lib.py) against include/kmpc.h's #defines."""
    from koopman_mpc_portfolio_rebalancing_amd import _lib
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "kmpc.h")).read()
    defs = {k: int(v) for k, v in re.findall(r"#define\s+(KMPC_\w+)\s+(-?\d+)\b", hdr)}
    assert defs["KMPC_PRECISION_AUTO"] == _lib.PRECISION_AUTO
    assert defs["KMPC_PRECISION_F64"] == _lib.PRECISION_F64
    assert defs["KMPC_PRECISION_MIXED"] == _lib.PRECISION_MIXED
    assert defs["KMPC_MIXED_MIN_B"] == _lib.MIXED_MIN_B
    assert defs["KMPC_PACK_MIN_B"] == _lib.PACK_MIN_B
    assert defs["KMPC_DTYPE_F32"] == _lib.DTYPE["fp32"]
    assert defs["KMPC_DTYPE_BF16"] == _lib.DTYPE["bf16"]
    assert defs["KMPC_DTYPE_F32_F32MFMA"] == _lib.DTYPE["fp32_f32mfma"]
    assert defs["KMPC_LATENT_AUTO"] == _lib.LATENT_FORM["auto"]
    assert defs["KMPC_LATENT_UNFUSED"] == _lib.LATENT_FORM["unfused"]
    assert defs["KMPC_LATENT_SEQUENTIAL"] == _lib.LATENT_FORM["sequential"]


def test_oracle_and_kernels_share_the_iteration_constants():
    """The kernels run the oracle's iteration: the initial multipliers, the no-short
    step factor and the capped-sigma bound are the same numbers in kmpc_solve_kernel.h and
    oracle/kmpc_oracle.c (the device's iteration counts track the oracle's, test_solver_gpu.py)."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hdr = open(os.path.join(root, "koopman_mpc_portfolio_rebalancing_amd", "csrc", "kmpc_solve_kernel.h")).read()
    orc = open(os.path.join(root, "oracle", "kmpc_oracle.c")).read()
    for name in ("KMPC_INIT_MULT", "KMPC_SIGMA_CAP", "KMPC_STEP_NOSHORT"):
        k = float(re.search(r"#define %s ([0-9.e-]+)" % name, hdr).group(1))
        o = float(re.search(r"#define %s R_\(([0-9.e-]+)\)" % name, orc).group(1))
        assert k == o, (name, k, o)
